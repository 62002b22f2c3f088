#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run18
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py -q > $O/pytest_fp8.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest_fp8.log; ok $rc || exit $rc
timeout -k 10 300 python tools/bench_gemm.py --json $O/bench_gemm.json > $O/bench_gemm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model gpt2_small --fp8 --steps 20 --warmup 5 > $O/bench_gpt2_fp8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet152 --steps 10 --warmup 5 > $O/bench_r152.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet152 --fp8 --steps 10 --warmup 5 > $O/bench_r152_fp8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --fp8 --steps 20 --warmup 8 > $O/bench_r50_fp8.log 2>&1 || exit $?
