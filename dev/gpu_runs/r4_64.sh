#!/bin/bash
# 1x1 conv weight gradients on the side stream: persistent ping-pong grid capped at 128 / 192 blocks vs one per CU
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_64
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad or gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for cap in 0 128 192; do
    PDNN_AB_PPCAP=$cap timeout -k 10 300 python3 -u bench.py --no-ddp-rehearsal --steps 20 --warmup 8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[cap=$cap] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
