#!/bin/bash
# dispatch-table sweep on the ResNet-50 step (PDNN_TUNE), same box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_12
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for T in "" "pp_conv_fwd_k=1024" "pp_conv_bnb_k=1024" "pp_conv_fwd_k=1024,pp_conv_bnb_k=1024" "lowk_bn64=8" "pp_conv_fwd_k=1024,pp_conv_bnb_k=1024,pp_conv_dgrad_k=1024" ""; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "$T $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
