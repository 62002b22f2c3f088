#!/bin/bash
# halo-kernel PRE staging with the BN-backward coefficients in LDS (more operand loads in flight): numerics, kernel
# timings (bf16 + fp8 dgrad), ResNet-50 same-box A/B vs HEAD base build
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_43
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_fp8_gpu.py -k "conv3x3" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 dev/probes/c3_fp8.py > $O/c3_fp8.jsonl 2>&1 || { cat $O/c3_fp8.jsonl; exit 1; }
cat $O/c3_fp8.jsonl
PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so timeout -k 10 120 python3 dev/probes/c3_fp8.py > $O/c3_fp8_base.jsonl 2>&1 || { cat $O/c3_fp8_base.jsonl; exit 1; }
cat $O/c3_fp8_base.jsonl
bash dev/probes/ab_lib.sh $O pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3 --steps 20 --warmup 8
