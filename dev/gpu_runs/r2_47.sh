#!/bin/bash
# round-end state (pp dgrad threshold 512): GPU suite, smoke, default bench, 1-rank RCCL DDP rehearsal, ResNet-152 bf16/fp8, GPT-2, kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_47
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 8; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -n 20 $O/smoke.log; exit 1; }
timeout -k 10 200 python -u bench.py > $O/bench_default.log 2>&1 && tail -n 1 $O/bench_default.log || exit 1
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/bench_r50_50.log 2>&1 && tail -n 1 $O/bench_r50_50.log | cut -c1-140 || exit 1
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29547 bench.py --gpus 1 --steps 30 --warmup 8 > $O/bench_ddp1.log 2>&1 && tail -n 1 $O/bench_ddp1.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --steps 10 --warmup 5 > $O/bench_r152.log 2>&1 && tail -n 1 $O/bench_r152.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --fp8 --steps 10 --warmup 5 > $O/bench_r152_fp8.log 2>&1 && tail -n 1 $O/bench_r152_fp8.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 30 --warmup 5 > $O/bench_gpt2.log 2>&1 && tail -n 1 $O/bench_gpt2.log | cut -c1-140 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo done
