#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run41
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn or block or model or graph or ddp" > $O/pytest.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_a.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_b.log 2>&1 || exit $?
