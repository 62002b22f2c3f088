#!/bin/bash
# fp8: trajectory test + fp8 suite, ResNet-152 bf16 / fp8 pair with the side-stream weight prefetch
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_38
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py tests/test_trajectory_gpu.py -k "fp8" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || { tail -20 $O/fp8_$i.err; exit 1; }
done
cut -c1-200 $O/*.json
