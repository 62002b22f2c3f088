#!/bin/bash
# deferred side-stream join: GPU suite, default bench (eager for ResNet), serial A/B, ResNet-152 bf16/fp8
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_33
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 8; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py > $O/bench_default$i.log 2>&1 && tail -n 1 $O/bench_default$i.log | cut -c1-140 || exit 1
done
PDNN_SIDE_WGRAD=0 timeout -k 10 200 python -u bench.py --graph off > $O/bench_serial_eager.log 2>&1 && tail -n 1 $O/bench_serial_eager.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --steps 10 --warmup 5 > $O/bench_r152.log 2>&1 && tail -n 1 $O/bench_r152.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --fp8 --steps 10 --warmup 5 > $O/bench_r152_fp8.log 2>&1 && tail -n 1 $O/bench_r152_fp8.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model resnet50 --fp8 > $O/bench_r50_fp8.log 2>&1 && tail -n 1 $O/bench_r50_fp8.log | cut -c1-140 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo done
