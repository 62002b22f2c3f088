#!/bin/bash
# host-side cost of the ResNet-50 step: small batches (GPU time small) expose the launch/Python time
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_28
mkdir -p $O
cd $GRAFT_REPO_ROOT
for B in 8 32 64 128 256; do
  timeout -k 10 200 python -u bench.py --batch $B --steps 20 --no-ddp-rehearsal > $O/b$B.log 2>&1 || exit 1
  echo "bs $B $(grep -o '"ms_per_step": [0-9.]*' $O/b$B.log)"
done
