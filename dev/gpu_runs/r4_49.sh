#!/bin/bash
# cross-entropy forward: cost of the per-row loss/count atomics
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_49
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 dev/probes/xent_probe.py > $O/xent.json 2>&1 || { cat $O/xent.json; exit 1; }
cat $O/xent.json
