#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run43
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small --fp8 > $O/gpt2_fp8.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small > $O/gpt2_bf16.log 2>&1 || exit $?
