#!/bin/bash
# split-K block target of the atomic conv weight gradients (stride-2 3x3, large 1x1): 512 (default) vs 256 / 1024
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_59
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash dev/probes/ab_bench.sh $O/a "wgrad_blocks=512" "wgrad_blocks=256" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/b "wgrad_blocks=512" "wgrad_blocks=1024" 2 --steps 20 --warmup 8 || exit 1
