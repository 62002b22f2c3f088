#!/bin/bash
# Fresh ResNet-50 bs256 kernel trace after the BN reduce specialisation
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run46
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1
