#!/bin/bash
# ResNet-50 1x1 weight gradients: long-reduction split model vs joint plan vs forced width x splits
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_36
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 dev/probes/wgrad1x1_sweep.py 2>&1 | grep -v amdgpu.ids | tee $O/sweep.txt || exit 1
echo done
