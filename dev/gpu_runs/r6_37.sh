#!/bin/bash
# GPT-2 kernel trace with the side-stream weight gradients: per-stream split
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_37
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g37 -o g37 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 5 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/g37.log 2>&1 || exit $?
find /tmp/g37 -name "*kernel_trace.csv" -exec cp {} $O/trace.csv \;
cd $R && python3 tools/stream_busy.py $O/trace.csv --step-kernel adam_kernel --full --top 25 > $O/streams.txt 2>&1
python3 tools/prof_summary.py $O/trace.csv --steps 3 --by-grid --top 40 > $O/grid_summary.txt 2>&1
cat $O/streams.txt | cut -c1-150
echo done
