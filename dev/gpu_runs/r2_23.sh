#!/bin/bash
# single-barrier pipelined pp main loop (PDNN_PP_PIPE=1) vs ping-pong: numerics, GEMM shapes, GPT-2 step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_23
mkdir -p $O
cd $GRAFT_REPO_ROOT
PDNN_PP_PIPE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or conv1x1" > $O/tests_pipe.log 2>&1 || { echo TESTS FAILED; tail -n 30 $O/tests_pipe.log; exit 1; }
tail -n 1 $O/tests_pipe.log
timeout -k 10 120 env PDNN_PP_PIPE=0 python -u tools/pp_check.py --perf-only > $O/g_p0.log 2>&1
timeout -k 10 120 env PDNN_PP_PIPE=1 python -u tools/pp_check.py --perf-only > $O/g_p1.log 2>&1
for P in 0 1; do
  for S in "8192 768 3072" "8192 3072 768" "8192 8192 8192"; do
    timeout -k 10 60 env PDNN_PP_PIPE=$P python -u tools/pp_one.py $S --bn 128 --trace --iters 10 2>&1 | grep -v amdgpu.ids | sed "s/^/pipe$P /" >> $O/trace.log || exit 1
  done
done
timeout -k 10 200 env PDNN_PP_PIPE=1 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2_p1.log 2>&1 && tail -n 1 $O/bench_gpt2_p1.log
echo done
