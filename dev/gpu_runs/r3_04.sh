#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_04
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_c3.log 2>&1
rc=$?; tail -n 5 $O/pytest_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_conv3x3.py > $O/bench_c3.log 2>&1 && cat $O/bench_c3.log || exit 1
bash dev/gpu_runs/r3_03.sh > $O/r3_03.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-150 || exit 1
echo done
