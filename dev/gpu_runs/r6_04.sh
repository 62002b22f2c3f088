#!/bin/bash
# determinism probe after the r6_03 rehearsal failure (per tuning setting), then the r6_03 A/B minus the failed test
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_04
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 dev/probes/s2_guard.py > $O/guard.log 2>&1 || { tail -30 $O/guard.log; exit 1; }
cat $O/guard.log | grep -v "^\[W\|amdgpu.ids"
timeout -k 10 300 python3 dev/probes/det_probe.py 30 s2_halo=0,ds_sub=0,side_wgrad=0 s2_halo=1,ds_sub=0,side_wgrad=0 s2_halo=0,ds_sub=0,side_wgrad=1 s2_halo=1,ds_sub=0,side_wgrad=1 > $O/det.log 2>&1 || { tail -30 $O/det.log; exit 1; }
cat $O/det.log | grep -v "^\[W\|amdgpu.ids"
echo done
