#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run25
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_r50 -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof_r50.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py /tmp/prof_r50/r50_kernel_trace.csv --window-ms 100 --steps 3 --top 25 > $O/r50_summary.txt
