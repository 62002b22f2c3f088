#!/bin/bash
# BN buffers as views of a flat tensor (DDP buffer broadcast without copy kernels): DDP tests, 1-rank RCCL bench, trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_38
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_fused_blocks_gpu.py tests/test_graphs_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2953$i bench.py --gpus 1 --steps 30 --warmup 8 > $O/bench_ddp1_$i.log 2>&1 && tail -n 1 $O/bench_ddp1_$i.log | cut -c1-140 || exit 1
done
cd /tmp && PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ddp --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo done
