#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run38
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 300 python bench.py > $O/base_$i.log 2>&1 || exit $?
  PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/gpurun_alt_libpdnn_kernels.so $T 300 python bench.py > $O/alt_$i.log 2>&1 || exit $?
done
