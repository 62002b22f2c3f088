#!/bin/bash
# ResNet-50 kernel trace after the r4 epilogue / BN / dgrad changes: per-grid breakdown + stream timeline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_21
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q4 -o q4 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-ddp-rehearsal > $O/q4.log 2>&1 || exit $?
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/q4_trace.csv \;
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $O/q4_trace.csv --steps 3 --by-grid --top 120 > $O/grid_summary.txt 2>&1
python3 tools/stream_timeline.py $O/q4_trace.csv --top 60 > $O/timeline.txt 2>&1
head -3 $O/grid_summary.txt; head -12 $O/timeline.txt
