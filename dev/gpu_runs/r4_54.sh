#!/bin/bash
# stem pooling passes: maxpool backward + BN reduce software-pipelined, BN-ReLU-maxpool one item per thread; A/B vs HEAD
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_54
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stem_gpu.py tests/test_kernels_gpu.py -k "pool or stem" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash dev/probes/ab_lib.sh $O/r50 pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3 --steps 20 --warmup 8 || exit 1
