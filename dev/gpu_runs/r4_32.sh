#!/bin/bash
# 1x1 stride-1 forwards (K >= 512, BN statistics) on the ping-pong engine: numerics, per-layer, same-box A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_32
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_tuning_gpu.py tests/test_conv1x1_wide_gpu.py tests/test_trajectory_gpu.py -k "not LeNet and not mlp and not ResNet18" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
PDNN_TUNE=pp_fwd1x1_k=1048576 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_off.log 2>&1 || { tail -20 $O/c1_off.log; exit 1; }
grep -h '"H"' $O/c1.log $O/c1_off.log | cut -c1-120
bash dev/probes/ab_bench.sh $O "pp_fwd1x1_k=512" "pp_fwd1x1_k=1048576" 3
