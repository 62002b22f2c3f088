#!/bin/bash
# side-stream weight-gradient grids, second pass: direct 3x3 wgrad 128 vs 64 blocks; + 1x1 split count x0.5
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_62
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash dev/probes/ab_bench.sh $O/a "w3_blocks=128" "w3_blocks=64" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/b "w3_blocks=128" "w3_blocks=128,wlong_scale=50" 3 --steps 20 --warmup 8 || exit 1
