#!/bin/bash
# per-layer cost of the masked residual and the BN-backward prologue on the 1x1 data gradients
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_18
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/l1x1.log 2>&1 || exit 1
cat $O/l1x1.log
