#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_08
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_fused_blocks_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/b1x1.log 2>&1 && cat $O/b1x1.log || exit 1
PDNN_PANEL1X1=0 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/b1x1_off.log 2>&1 && tail -n 1 $O/b1x1_off.log || exit 1
timeout -k 10 200 python -u bench.py --steps 30 > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-150 || exit 1
PDNN_PANEL1X1=0 timeout -k 10 200 python -u bench.py --steps 30 > $O/bench_off.log 2>&1 && tail -n 1 $O/bench_off.log | cut -c1-150 || exit 1
echo done
