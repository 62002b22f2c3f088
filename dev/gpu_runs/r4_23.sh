#!/bin/bash
# BN3 backward link (C3_RESBN epilogue): kernel test, flagship numerics, same-box A/B bn_link=1 vs 0
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_23
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
true


bash dev/probes/ab_bench.sh $O "bn_link=1" "bn_link=0" 3
