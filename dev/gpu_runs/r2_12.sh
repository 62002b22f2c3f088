#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_graphs_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o gpt2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1
