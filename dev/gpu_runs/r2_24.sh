#!/bin/bash
# validation after removing the pipelined experiment: kernel tests (all engines), forced pp fusions, benches
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_24
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
PDNN_PP_CONV_FWD_K=0 PDNN_PP_CONV_BNB=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/tests_ppfx.log 2>&1 || { echo FX TESTS FAILED; tail -n 30 $O/tests_ppfx.log; exit 1; }
tail -n 1 $O/tests_ppfx.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_r50.log 2>&1 && tail -n 1 $O/bench_r50.log
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 && tail -n 1 $O/bench_gpt2.log
echo done
