#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_05
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_fused_blocks_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-150 || exit 1
PDNN_MATERIALIZE_A2=0 timeout -k 10 200 python -u bench.py > $O/bench_pro.log 2>&1 && tail -n 1 $O/bench_pro.log | cut -c1-150 || exit 1
timeout -k 10 200 python -u bench.py --steps 40 > $O/bench40.log 2>&1 && tail -n 1 $O/bench40.log | cut -c1-150 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo done
