#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run19
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > $O/pytest_k.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest_k.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.log 2>&1 || exit $?
PDNN_STAGED_STORE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_direct.log 2>&1 || exit $?
PDNN_GLDS=0 timeout -k 10 400 python tools/bench_conv.py --no-ref --json $O/conv_staged.json > $O/conv_staged.log 2>&1 || exit $?
PDNN_GLDS=0 PDNN_STAGED_STORE=0 timeout -k 10 400 python tools/bench_conv.py --no-ref --json $O/conv_direct.json > $O/conv_direct.log 2>&1 || exit $?
