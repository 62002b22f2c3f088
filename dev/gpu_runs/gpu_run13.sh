#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run13
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -m pytest tests/test_transformer_gpu.py -q > $O/pytest_tx.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest_tx.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gpt2 -o gpt2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 3 --warmup 3 > $O/prof_gpt2.log 2>&1 || exit $?
