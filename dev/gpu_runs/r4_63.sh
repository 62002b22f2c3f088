#!/bin/bash
# weight-gradient grid changes: numerics of the affected kernels, then driver-style bench x2 and ResNet-152 pair
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_63
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_trajectory_gpu.py tests/test_fused_blocks_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 400 python3 bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  cut -c1-160 $O/bench_$i.json
done
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-110 $O/bf16_*.json $O/fp8_*.json
