#!/bin/bash
# GPT-2 small bs8 kernel breakdown with the current kernels (eager step, kernel trace + stats only)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run67
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1
