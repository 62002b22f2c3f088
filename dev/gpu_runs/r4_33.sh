#!/bin/bash
# 1x1 stride-1 forwards (K >= 512, BN statistics) on the ping-pong engine: numerics, per-layer, same-box A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_33
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash dev/probes/ab_bench.sh $O "pp_fwd1x1_k=1024" "pp_fwd1x1_k=1048576" 3
