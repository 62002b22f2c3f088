#!/bin/bash
# ResNet-50 kernel trace after the round-6 ping-pong / statistics changes: per-stream split with template names
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_23
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q23 -o q23 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --plain > $O/q.log 2>&1 || exit $?
find /tmp/q23 -name "*kernel_trace.csv" -exec cp {} $O/trace.csv \;
cd $R && python3 tools/prof_summary.py $O/trace.csv --steps 3 --by-grid --top 80 > $O/grid_summary.txt 2>&1
python3 tools/stream_busy.py $O/trace.csv --full --top 40 > $O/streams.txt 2>&1
head -3 $O/grid_summary.txt
cat $O/streams.txt | cut -c1-160
echo done
