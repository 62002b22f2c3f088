#!/bin/bash
# GPT-2 weight-gradient GEMMs: tile width x K-split sweep
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_33
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 dev/probes/wgrad_sweep.py 2>&1 | grep -v amdgpu.ids | tee $O/sweep.txt || exit 1
echo done
