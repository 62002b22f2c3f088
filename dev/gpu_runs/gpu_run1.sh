#!/bin/bash
# GPU run 1: stock PyTorch-ROCm ResNet-50 comparison line + kernel breakdown.
set -o pipefail
mkdir -p gpurun_out/run1
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/run1/smi.txt 2>&1 || true
for mode in bf16 autocast; do
  timeout -k 10 300 python tools/stock_baseline.py --mode $mode --batch 256 --steps 15 --warmup 5 >> gpurun_out/run1/stock.jsonl 2>> gpurun_out/run1/stock.err || exit $?
done
timeout -k 10 200 python tools/stock_baseline.py --mode bf16 --batch 128 --steps 15 --warmup 5 >> gpurun_out/run1/stock.jsonl 2>> gpurun_out/run1/stock.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/run1/prof -o stock --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stock_baseline.py --mode bf16 --batch 256 --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/run1/prof.log 2>&1
