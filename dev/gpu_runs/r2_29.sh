#!/bin/bash
# GPT-2 --fp8 kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_29
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o gpt2fp8 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --fp8 --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1
echo done
