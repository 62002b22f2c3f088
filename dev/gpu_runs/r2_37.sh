#!/bin/bash
# side-aware DDP bucket launches: DDP tests, full suite, 1-rank RCCL DDP bench rehearsal vs plain
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_37
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 8; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2953$i bench.py --gpus 1 --steps 30 --warmup 8 > $O/bench_ddp1_$i.log 2>&1 && tail -n 1 $O/bench_ddp1_$i.log | cut -c1-140 || exit 1
done
timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-140 || exit 1
echo done
