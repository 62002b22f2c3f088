#!/bin/bash
# fp8 status: GPT-2 and ResNet-152 with and without --fp8; GPT-2 kernel trace (bf16) after the wgrad change
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_27
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py --model gpt2_small --fp8 --steps 20 --warmup 5 > $O/gpt2_fp8.log 2>&1; tail -n 1 $O/gpt2_fp8.log
timeout -k 10 300 python -u bench.py --model resnet152 --steps 10 --warmup 3 > $O/r152.log 2>&1; tail -n 1 $O/r152.log
timeout -k 10 300 python -u bench.py --model resnet152 --fp8 --steps 10 --warmup 3 > $O/r152_fp8.log 2>&1; tail -n 1 $O/r152_fp8.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o gpt2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1
echo done
