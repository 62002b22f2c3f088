#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run17
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/ -q -m gpu > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gemm.py --json $O/bench_gemm.json > $O/bench_gemm.log 2>&1 || exit $?
