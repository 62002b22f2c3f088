#!/bin/bash
# ResNet-152 bf16 / fp8 same-box pairs after the LDS-coefficient staging
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_44
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-200 $O/*.json
cd /tmp
export TMPDIR=/tmp
cut -c1-120 $O/*.json
