#!/bin/bash
# One-launch (last-block) BN slab finalize A/B vs the two-launch path (measured slower; superseded by run49)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run47
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  $T 200 python bench.py > $O/bench_fused_$rep.log 2>&1 || exit $?
  PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/build/alt/lib_nofin.so $T 200 python bench.py > $O/bench_nofin_$rep.log 2>&1 || exit $?
done
$T 200 python bench.py --graph on > $O/bench_fused_graph.log 2>&1 || exit $?
