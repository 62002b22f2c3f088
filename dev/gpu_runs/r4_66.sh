#!/bin/bash
# BN apply / BN-backward apply grid cap, lower end: 1024 / 768 / 512 / 256 blocks
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_66
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "bn or batchnorm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for cap in 1024 768 512 256; do
    PDNN_AB_BNGRID=$cap timeout -k 10 300 python3 -u bench.py --no-ddp-rehearsal --steps 20 --warmup 8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[bngrid=$cap] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
