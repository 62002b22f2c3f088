#!/bin/bash
# dispatch-table re-sweep on the end-state build: 128x64 tile threshold, BN-fused dgrads on the ping-pong engine
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_70
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for T in "" "lowk_bn64=8" "lowk_bn64=16" "lowk_bn64=32" "pp_conv_bnb_k=512" "pp_conv_bnb_k=1024" "" "lowk_bn64=8" "pp_conv_bnb_k=512"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
