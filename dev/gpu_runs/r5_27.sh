#!/bin/bash
# fused cross-entropy: per-step GPT-2 losses, on / off, twice each
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_27
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 dev/probes/xent_traj.py --ddp > $O/traj_ddp.txt 2>&1; cat $O/traj_ddp.txt | grep -v amdgpu.ids
