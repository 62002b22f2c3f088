#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run11
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k colsum > $O/pytest_colsum.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest_colsum.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
timeout -k 10 400 python tools/gpt2_check.py > $O/gpt2_check.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_gemm.py --json $O/bench_gemm.json > $O/bench_gemm.log 2>&1 || exit $?
