#!/bin/bash
# hipGraph step vs eager A/B on the current kernels (ResNet-50 bs256, GPT-2 small bs8), and the
# single-rank RCCL DDP rehearsal (forced bucket all-reduces) after the clean rebuild
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run60
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for rep in 1 2; do
  for g in off auto; do
    $T 200 python -u bench.py --steps 20 --warmup 5 --graph $g > $O/r50_${g}_$rep.log 2>&1 || exit $?
    $T 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 --graph $g > $O/gpt2_${g}_$rep.log 2>&1 || exit $?
  done
done
export PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1
$T 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 > $O/bench_rccl1.log 2>&1 || exit $?
$T 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --model gpt2_small > $O/bench_rccl1_gpt2.log 2>&1 || exit $?
