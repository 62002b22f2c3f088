#!/bin/bash
# direct 3x3 wgrad timing ablations
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_44
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/w3_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
