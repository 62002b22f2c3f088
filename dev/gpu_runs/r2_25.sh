#!/bin/bash
# tied-wte direct arena accumulation: transformer tests + GPT-2 bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_25
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 && tail -n 1 $O/bench_gpt2.log
echo done
