#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run33
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -v --timeout 120 --timeout-method thread -k "colsum or adam or sgd or xent" > $O/pytest.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
cd /tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_g2 -o g2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 4 --warmup 3 > $O/prof_g2.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py /tmp/prof_g2/g2_kernel_trace.csv --window-ms 52 --steps 3 --top 40 > $O/g2_summary.txt
