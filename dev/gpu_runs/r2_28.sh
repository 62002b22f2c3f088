#!/bin/bash
# fp8 on the ping-pong engine: numerics (both engines), GEMM shapes, GPT-2 / ResNet-152 --fp8 steps
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_28
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python -u tools/bench_gemm.py --json $O/gemm_pp.json > $O/gemm_pp.log 2>&1; grep -v amdgpu $O/gemm_pp.log | head -12
timeout -k 10 200 env PDNN_PP_FP8=0 python -u tools/bench_gemm.py --json $O/gemm_glds.json > $O/gemm_glds.log 2>&1; grep -v amdgpu $O/gemm_glds.log | head -12
timeout -k 10 200 python -u bench.py --model gpt2_small --fp8 --steps 20 --warmup 5 > $O/gpt2_fp8.log 2>&1; tail -n 1 $O/gpt2_fp8.log
timeout -k 10 300 python -u bench.py --model resnet152 --fp8 --steps 10 --warmup 3 > $O/r152_fp8.log 2>&1; tail -n 1 $O/r152_fp8.log
echo done
