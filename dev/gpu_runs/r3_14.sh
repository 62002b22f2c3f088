#!/bin/bash
# bench A/B of the fused BN-backward operand prologue (tuning bwd_pre), same box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_14
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for T in "" "bwd_pre=0" "" "bwd_pre=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
