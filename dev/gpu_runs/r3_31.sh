#!/bin/bash
# secondary benches: ResNet-152 bf16 vs fp8, GPT-2 small in-tree GEMMs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_31
mkdir -p $O
cd $GRAFT_REPO_ROOT
for args in "--model resnet152" "--model resnet152 --fp8" "--model resnet152" "--model resnet152 --fp8" "--model gpt2_small" "--model gpt2_small --fp8"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -u bench.py $args --steps 20 --no-ddp-rehearsal > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$args $(grep -o '"value": [0-9.]*' $O/$n.log)"
done
