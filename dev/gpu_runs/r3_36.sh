#!/bin/bash
# kernel traces with and without the identity-block BN hand-off
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_36
mkdir -p $O
cd /tmp
for T in "bn_link=1" "bn_link=0"; do
  PDNN_TUNE="$T" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof_$T.log 2>&1 || exit 1
done
echo done
