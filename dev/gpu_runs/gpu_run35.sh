#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run35
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "dgrad or block or model" > $O/pytest.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_r50_a.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_r50_b.log 2>&1 || exit $?
