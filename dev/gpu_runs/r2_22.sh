#!/bin/bash
# conv numerics with the new routing defaults; ResNet-50 and GPT-2 benches; GPT-2 kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_22
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_r50.log 2>&1 && tail -n 1 $O/bench_r50.log
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 && tail -n 1 $O/bench_gpt2.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o gpt2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1
echo done
