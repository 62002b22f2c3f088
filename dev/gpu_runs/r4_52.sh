#!/bin/bash
# BN1 + ReLU applied while staging (fuse_a1): ResNet-50 same-box A/B against the materialised a1, ResNet-152 pairs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_52
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash dev/probes/ab_bench.sh $O/r50 "fuse_a1=0" "fuse_a1=1" 3 --steps 20 --warmup 8 || exit 1
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-110 $O/*.json
