#!/bin/bash
# wgrad split cost model: GEMM shapes + GPT-2 step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_26
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/pp_check.py --perf-only > $O/g.log 2>&1 && grep wg_ $O/g.log
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 && tail -n 1 $O/bench_gpt2.log
echo done
