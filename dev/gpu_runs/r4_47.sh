#!/bin/bash
# fp8 direct 3x3 weight gradient: numerics, timing vs bf16, ResNet-152 bf16 / fp8 pair
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_47
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -k "wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python3 dev/probes/w8_bench.py > $O/w8.jsonl 2>&1 || { cat $O/w8.jsonl; exit 1; }
cat $O/w8.jsonl
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_trajectory_gpu.py -k fp8 > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
tail -2 $O/traj.log
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-110 $O/*.json
