#!/bin/bash
# straggler kill on the GPU, bench with the DDP-path rehearsal, k-of-n throttle cost, RCCL floor table,
# rocprof of the 1-rank RCCL rehearsal
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_09
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_straggler_gpu.py tests/test_tuning_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_strag.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest_strag.log | tail -n 8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 > $O/bench.log 2>&1 && tail -n 1 $O/bench.log || exit 1
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 $R --master-port 29611 bench.py --gpus 1 --steps 30 --warmup 8 > $O/bench_ddp1.log 2>&1 && tail -n 1 $O/bench_ddp1.log | cut -c1-150 || exit 1
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 $R --master-port 29612 bench.py --gpus 1 --steps 30 --warmup 8 --num-aggregate 1 > $O/bench_kofn1.log 2>&1 && tail -n 1 $O/bench_kofn1.log | cut -c1-150 || exit 1
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 $R --master-port 29613 bench.py --gpus 1 --steps 30 --warmup 8 --comm-bf16 > $O/bench_bf16wire.log 2>&1 && tail -n 1 $O/bench_bf16wire.log | cut -c1-150 || exit 1
PDNN_FORCE_PG=1 timeout -k 10 300 $R --master-port 29614 tools/bench_allreduce.py --ops all_reduce,broadcast --dtypes float32,bfloat16 > $O/allreduce_w1.log 2>&1 && grep '^{' $O/allreduce_w1.log | tail -n 4 || exit 1
cd /tmp && PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29615 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ddp1 -o ddp1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof_ddp1.log 2>&1 || exit 1
echo done
