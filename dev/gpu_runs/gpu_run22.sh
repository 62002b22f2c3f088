#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run22
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_r50 -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof_r50.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py /tmp/prof_r50/r50_kernel_trace.csv --window-ms 100 --steps 3 --top 40 > $O/r50_summary.txt
cp /tmp/prof_r50/r50_kernel_stats.csv $O/
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_stock -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stock_baseline.py --mode autocast --steps 3 --warmup 3 > $O/prof_stock.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py /tmp/prof_stock/st_kernel_trace.csv --window-ms 115 --steps 3 --top 40 > $O/stock_summary.txt
