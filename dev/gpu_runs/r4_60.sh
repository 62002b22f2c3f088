#!/bin/bash
# split-K block target of the atomic conv weight gradients: 256 vs 128 / 384
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_60
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash dev/probes/ab_bench.sh $O/a "wgrad_blocks=256" "wgrad_blocks=128" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/b "wgrad_blocks=256" "wgrad_blocks=384" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/c "wgrad_blocks=512" "wgrad_blocks=256" 2 --steps 20 --warmup 8 || exit 1
