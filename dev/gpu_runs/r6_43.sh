#!/bin/bash
# GPT-2 kernel trace after wgrad_plan_cus=128: per-stream split and side-kernel overlap of the attention backward
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_43
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g43 -o g43 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 5 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/g43.log 2>&1 || exit $?
find /tmp/g43 -name "*kernel_trace.csv" -exec cp {} $O/trace.csv \;
cd $R && python3 tools/stream_busy.py $O/trace.csv --step-kernel adam_kernel --full --top 25 > $O/streams.txt 2>&1
python3 tools/prof_summary.py $O/trace.csv --steps 3 --by-grid --top 40 > $O/grid_summary.txt 2>&1
cat $O/streams.txt | cut -c1-150
echo done
