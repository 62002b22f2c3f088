#!/bin/bash
# Adam kernel software-pipelined (next element's loads before this element's stores): numerics + GPT-2 A/B vs HEAD
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_48
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_graphs_gpu.py -k "adam or optim or gpt" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash dev/probes/ab_lib.sh $O/gpt pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3 --model gpt2_small --steps 20 --warmup 8 || exit 1
