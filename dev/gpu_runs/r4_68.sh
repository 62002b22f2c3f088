#!/bin/bash
# generic streaming-kernel grid cap (elementwise, pooling, optimizer, slab reduces): 2048 (current) / 1024 / 512,
# with the BN apply kernels fixed at 512; ResNet-50 and GPT-2
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_68
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for cap in 2048 1024 512; do
    PDNN_AB_SGRID=$cap timeout -k 10 300 python3 -u bench.py --no-ddp-rehearsal --steps 20 --warmup 8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[resnet50 sgrid=$cap] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
for i in 1 2; do
  for cap in 2048 512; do
    PDNN_AB_SGRID=$cap timeout -k 10 300 python3 -u bench.py --model gpt2 --no-ddp-rehearsal --steps 20 --warmup 8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[gpt2 sgrid=$cap] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
