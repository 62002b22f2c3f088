#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run36
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
$T 200 python tools/bench_attn.py > $O/attn.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small > $O/bench_gpt2.log 2>&1 || exit $?
