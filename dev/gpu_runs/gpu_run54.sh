#!/bin/bash
# maxpool (32-bit indices, templated 3x3 window) + vectorized NCHW->NHWC: numerics, bench, trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run54
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
$T 200 python bench.py > $O/bench_1.log 2>&1 || exit $?
$T 200 python bench.py > $O/bench_2.log 2>&1 || exit $?
cd /tmp && $T 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1
