#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run14
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/ -q -m gpu > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r50 -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof_r50.log 2>&1 || exit $?
