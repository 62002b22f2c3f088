#!/bin/bash
# dispatch-table re-sweep under the current kernels (one process per setting, interleaved rounds)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_41
mkdir -p $O
cd $GRAFT_REPO_ROOT
i=0
for round in 1 2; do
for T in "" "pp_conv_bnb_k=512" "glds_dgrad_k=512" "lowk_bn64=16" "lowk_bn64=32" "split_blocks=768" "pp_conv_fwd_k=512" "glds_fwd_k=512"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
done
echo done
