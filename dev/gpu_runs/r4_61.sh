#!/bin/bash
# side-stream weight-gradient grid sizes in the two-stream schedule: direct 3x3 wgrad block target (256 default vs
# 128 / 512) and the 1x1 long-reduction split count (x0.5 / x2)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_61
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash dev/probes/ab_bench.sh $O/a "w3_blocks=256" "w3_blocks=128" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/b "w3_blocks=256" "w3_blocks=512" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/c "wlong_scale=100" "wlong_scale=50" 2 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_bench.sh $O/d "wlong_scale=100" "wlong_scale=200" 2 --steps 20 --warmup 8 || exit 1
