#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run16
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > $O/pytest_k.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest_k.log; ok $rc || exit $rc
timeout -k 10 600 python -m pytest tests/ -q -m gpu --deselect tests/test_kernels_gpu.py > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_conv.py --no-ref --json $O/conv.json > $O/conv.log 2>&1 || exit $?
PDNN_GLDS=0 timeout -k 10 400 python tools/bench_conv.py --no-ref --json $O/conv_reg.json > $O/conv_reg.log 2>&1 || exit $?
