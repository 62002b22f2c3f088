#!/bin/bash
# BN statistics / BN-backward reduce grids around r4_70 optimum: cap 512 / 384, min rows per thread row 64 / 32
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_71
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "bn or batchnorm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for cr in 512:64 512:32 384:64 384:32; do
    PDNN_AB_RCAP=${cr%:*} PDNN_AB_RMIN=${cr#*:} timeout -k 10 300 python3 -u bench.py --no-ddp-rehearsal --steps 20 --warmup 8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[rcap:rmin=$cr] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
