#!/bin/bash
# BN grid caps split: forward BN apply (F) vs backward BN apply (B), around the 512 optimum of r4_66
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_67
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for fb in 512:512 2048:512 512:2048 512:384 384:512 1024:512; do
    PDNN_AB_BNF=${fb%:*} PDNN_AB_BNB=${fb#*:} timeout -k 10 300 python3 -u bench.py --no-ddp-rehearsal --steps 20 --warmup 8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[F:B=$fb] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
