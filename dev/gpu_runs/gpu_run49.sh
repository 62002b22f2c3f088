#!/bin/bash
# Wide-grid two-launch BN slab finalize: numerics + ResNet-50 A/B against the two-launch path (PDNN_BN_WIDE_FIN=0)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run49
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  $T 200 python bench.py > $O/bench_fused_$rep.log 2>&1 || exit $?
  PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/build/alt/lib_nofin.so $T 200 python bench.py > $O/bench_nofin_$rep.log 2>&1 || exit $?
done
$T 200 python bench.py --graph on > $O/bench_fused_graph.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1
