#!/bin/bash
# RCCL path rehearsal on one GPU: 1-rank nccl process group with DDP communication forced on
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run50
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
export PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1
$T 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 > $O/bench_rccl1.log 2>&1 || exit $?
$T 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --bucket-mb 8 > $O/bench_rccl1_b8.log 2>&1 || exit $?
unset PDNN_FORCE_PG PDNN_DDP_FORCE_COMM
$T 200 python bench.py > $O/bench_plain.log 2>&1 || exit $?
