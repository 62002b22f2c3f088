#!/bin/bash
# GPT-2 small kernel breakdown, end of round 4
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_56
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g5 -o g5 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 4 --warmup 2 --no-ddp-rehearsal --graph off > $O/g5.log 2>&1 || exit $?
find /tmp/g5 -name "*kernel_trace.csv" -exec cp {} $O/g5_trace.csv \;
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $O/g5_trace.csv --steps 3 --by-grid --top 40 > $O/g5_summary.txt 2>&1
head -30 $O/g5_summary.txt | cut -c1-170
