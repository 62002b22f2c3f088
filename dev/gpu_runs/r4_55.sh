#!/bin/bash
# cross-entropy backward: next chunks' loads before this chunk's stores; xent timing + GPT-2 A/B vs HEAD
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_55
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_gpu.py -k "xent or gpt" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 dev/probes/xent_probe.py > $O/xent.json 2>&1 || { cat $O/xent.json; exit 1; }
cat $O/xent.json
PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so timeout -k 10 120 python3 dev/probes/xent_probe.py > $O/xent_base.json 2>&1 || { cat $O/xent_base.json; exit 1; }
cat $O/xent_base.json
bash dev/probes/ab_lib.sh $O/gpt pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3 --model gpt2_small --steps 20 --warmup 8 || exit 1
