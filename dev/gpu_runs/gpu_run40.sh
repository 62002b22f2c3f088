#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run40
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_r50 -o r50 --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $O/prof_r50.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py /tmp/prof_r50/r50_kernel_trace.csv --window-ms 105 --steps 3 --top 40 > $O/r50_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_g2 -o g2 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 4 --warmup 3 > $O/prof_g2.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py /tmp/prof_g2/g2_kernel_trace.csv --window-ms 50 --steps 3 --top 40 > $O/g2_summary.txt
