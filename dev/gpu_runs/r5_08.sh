#!/bin/bash
# GPT-2 small after the attention block order: kernel trace breakdown (DDP path, eager)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_08
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g4 -o g4 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g4.log 2>&1 || exit $?
find /tmp/g4 -name "*kernel_trace.csv" -exec cp {} $O/g4_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g4_trace.csv --steps 3 --by-grid --top 50 > $O/grid_summary.txt 2>&1
head -45 $O/grid_summary.txt
