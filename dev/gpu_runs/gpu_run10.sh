#!/bin/bash
# stock GPT-2 line + kernel profiles of our GPT-2 and ResNet-50 steps
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/stock_gpt2.py --steps 10 --warmup 3 > $O/stock_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model gpt2_small --steps 30 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/bench.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gpt2 -o gpt2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 3 --warmup 3 > $O/prof_gpt2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r50 -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof_r50.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stock_gpt2 -o sg --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stock_gpt2.py --steps 3 --warmup 3 > $O/prof_stock_gpt2.log 2>&1 || exit $?
