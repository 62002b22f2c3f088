#!/bin/bash
# A/B: ResNet weight gradients on a side stream (PDNN_SIDE_WGRAD=1, default) vs serial; GPU suite
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_32
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
PDNN_SIDE_WGRAD=0 timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 > $O/bench_serial$i.log 2>&1 && tail -n 1 $O/bench_serial$i.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 > $O/bench_side$i.log 2>&1 && tail -n 1 $O/bench_side$i.log | cut -c1-140 || exit 1
done
timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 --graph off > $O/bench_side_eager.log 2>&1 && tail -n 1 $O/bench_side_eager.log | cut -c1-140 || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --steps 10 --warmup 5 > $O/bench_r152.log 2>&1 && tail -n 1 $O/bench_r152.log | cut -c1-140 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1 || exit 1
echo done
