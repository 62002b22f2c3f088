#!/bin/bash
# host vs GPU: kernel trace + HIP runtime API trace of the ResNet-50 step (when each launch was issued)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_66
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
ls $O/prof
echo done
