#!/bin/bash
# DDP forced-communication drift diagnosis (nccl / gloo / no comm) on one GPU
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run51
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
P=29620
for mode in nocomm gloo nccl; do
  P=$((P+1))
  $T 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P tools/ddp_diag.py $mode > $O/diag_$mode.log 2>&1 || exit $?
done
P=$((P+1))
DIAG_LR=0 $T 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P tools/ddp_diag.py nocomm > $O/diag_nocomm_lr0.log 2>&1 || exit $?
