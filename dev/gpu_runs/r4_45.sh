#!/bin/bash
# split-K slab reduces: tail splits as 4/2/1 loads issued together; numerics + ResNet-50 / GPT-2 same-box A/B vs HEAD
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_45
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_tuning_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash dev/probes/ab_lib.sh $O/r50 pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3 --steps 20 --warmup 8 || exit 1
bash dev/probes/ab_lib.sh $O/gpt pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 2 --model gpt2_small --steps 20 --warmup 8 || exit 1
