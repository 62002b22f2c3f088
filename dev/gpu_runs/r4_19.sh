#!/bin/bash
# BatchNorm apply kernels software-pipelined across rows: numerics, per-layer, same-box A/B vs HEAD
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_19
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv3x3_gpu.py tests/test_stem_gpu.py tests/test_trajectory_gpu.py tests/test_models_gpu.py -k "not ResNet18 and not LeNet and not mlp" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
tail -1 $O/c1.log | cut -c1-400
PDNN_KERNEL_LIB=pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_base.log 2>&1 || { tail -20 $O/c1_base.log; exit 1; }
tail -1 $O/c1_base.log | cut -c1-400
bash dev/probes/ab_lib.sh $O pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3
