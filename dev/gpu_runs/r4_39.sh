#!/bin/bash
# fp8 dgrad staging in two 8-channel passes (8 loads in flight); no bf16 flip for fp8 blocks
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_39
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py -k conv3x3 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 dev/probes/c3_fp8.py > $O/c3_fp8.jsonl 2>&1 || { cat $O/c3_fp8.jsonl; exit 1; }
cat $O/c3_fp8.jsonl
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || { tail -20 $O/fp8_$i.err; exit 1; }
done
cut -c1-200 $O/*.json
