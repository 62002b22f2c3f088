#!/bin/bash
# 1x1 K>=512 data gradients with the BN-backward epilogue on the ping-pong engine (t prefetched a row ahead)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_16
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv1x1_wide_gpu.py tests/test_tuning_gpu.py tests/test_trajectory_gpu.py -k "not ResNet18 and not LeNet and not mlp" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
grep -v amdgpu $O/c1.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-ddp-rehearsal > $O/r50.log 2>&1 || { tail -20 $O/r50.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r50.log
