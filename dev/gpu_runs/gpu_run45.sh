#!/bin/bash
# BN streaming kernels A/B: reduce unroll (UR), apply unroll (UA), reduce min rows/thread (RMIN)
# A: UR2 UA2 RMIN64 | B: UR2 UA2 RMIN16 | C: UR1 UA2 RMIN16 | D: UR4 UA2 RMIN16 | E: UR2 UA1 RMIN64
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run45
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
A=$GRAFT_REPO_ROOT/build/alt
PDNN_KERNEL_LIB=$A/lib_D.so $T 300 python -u -m pytest tests/test_fused_blocks_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_D.log 2>&1 || exit $?
for rep in 1 2; do for V in A B C D E; do
  PDNN_KERNEL_LIB=$A/lib_$V.so $T 200 python bench.py > $O/bench_${V}_$rep.log 2>&1 || exit $?
done; done
