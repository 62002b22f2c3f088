#!/bin/bash
# GPT-2 small kernel trace with the paired / slack ping-pong epilogues (profile), plus a per-stream split
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_14
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g14 -o g14 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 5 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/g14.log 2>&1 || exit $?
find /tmp/g14 -name "*kernel_trace.csv" -exec cp {} $O/g14_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g14_trace.csv --steps 3 --by-grid --top 60 > $O/grid_summary.txt 2>&1
python3 tools/stream_busy.py $O/g14_trace.csv --step-kernel adam_kernel --top 20 > $O/streams.txt 2>&1
head -40 $O/grid_summary.txt
cat $O/streams.txt
echo done
