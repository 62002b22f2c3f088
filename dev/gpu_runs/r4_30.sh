#!/bin/bash
# implicit-GEMM gathers resolved per tap (not per K-step): numerics (conv kernels, stem, tuning battery, flagship),
# strided data gradients, per-layer convs, same-box A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_30
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_tuning_gpu.py tests/test_stem_gpu.py tests/test_fused_blocks_gpu.py tests/test_trajectory_gpu.py tests/test_models_gpu.py -k "not LeNet and not mlp" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u dev/probes/strided_dgrad.py > $O/sd.log 2>&1 || { tail -20 $O/sd.log; exit 1; }
PDNN_KERNEL_LIB=pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so timeout -k 10 200 python -u dev/probes/strided_dgrad.py > $O/sd_base.log 2>&1 || { tail -20 $O/sd_base.log; exit 1; }
tail -1 $O/sd.log; tail -1 $O/sd_base.log
bash dev/probes/ab_lib.sh $O pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3
