#!/bin/bash
# refresh secondary configs: GPT-2 small bf16/fp8, ResNet-152 bf16/fp8; trace of the ResNet-152 fp8 step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run56
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python bench.py --model gpt2_small > $O/gpt2_bf16.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small --fp8 > $O/gpt2_fp8.log 2>&1 || exit $?
$T 300 python bench.py --model resnet152 --steps 10 --warmup 5 > $O/r152_bf16.log 2>&1 || exit $?
$T 300 python bench.py --model resnet152 --steps 10 --warmup 5 --fp8 > $O/r152_fp8.log 2>&1 || exit $?
cd /tmp && $T 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r152fp8 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet152 --fp8 --steps 2 --warmup 3 > $O/prof.log 2>&1
