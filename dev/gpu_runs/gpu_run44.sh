#!/bin/bash
# BN streaming kernels: rows-per-iteration A/B (PDNN_BN_U = 2 / 4 / 8) on the ResNet-50 step + numerics
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run44
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
A=$GRAFT_REPO_ROOT/build/alt
for U in 8 4; do
  PDNN_KERNEL_LIB=$A/libpdnn_kernels_u$U.so $T 300 python -u -m pytest tests/test_fused_blocks_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_u$U.log 2>&1 || exit $?
done
for rep in 1 2; do for U in 2 4 8; do
  PDNN_KERNEL_LIB=$A/libpdnn_kernels_u$U.so $T 200 python bench.py > $O/bench_u${U}_$rep.log 2>&1 || exit $?
done; done
