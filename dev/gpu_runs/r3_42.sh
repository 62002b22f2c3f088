#!/bin/bash
# per-layer weight-gradient timings: default routing, forced glds, MIOpen reference
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_42
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/bench_conv.py --only wgrad --json $O/wg_default.json > $O/wg_default.log 2>&1 || { tail -20 $O/wg_default.log; exit 1; }
grep -v amdgpu.ids $O/wg_default.log | tail -30
PDNN_TUNE="glds=2" timeout -k 10 400 python -u tools/bench_conv.py --only wgrad --no-ref --json $O/wg_glds.json > $O/wg_glds.log 2>&1 || { tail -20 $O/wg_glds.log; exit 1; }
grep -v amdgpu.ids $O/wg_glds.log | tail -30
echo done
