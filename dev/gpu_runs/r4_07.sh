#!/bin/bash
# flagship first-step gradient agreement per layer group vs stock fp32 at several residual-branch gains
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_07
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for g in 0.3 0.1; do
timeout -k 10 300 python -u dev/probes/grad_cos.py --bn3 $g > $O/cos_112_$g.log 2>&1 || { tail -20 $O/cos_112_$g.log; exit 1; }
grep -v amdgpu.ids $O/cos_112_$g.log
done
