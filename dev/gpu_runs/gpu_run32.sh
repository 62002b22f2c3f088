#!/bin/bash
# GPT-2 linears: hipBLASLt GEMM cores (auto) vs in-tree MFMA; numerics + bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run32
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_graphs_gpu.py -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PDNN_GEMM=mfma $T 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2_mfma.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2_auto.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small --steps 20 --warmup 5 --graph on > $O/bench_gpt2_auto_graph.log 2>&1 || exit $?
