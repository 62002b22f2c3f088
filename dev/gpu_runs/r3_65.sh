#!/bin/bash
# secondary benches on the end-state build: ResNet-152 bf16 vs fp8 weights, GPT-2 bf16 vs fp8
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_65
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for M in "--model resnet152" "--model resnet152 --fp8" "--model resnet152" "--model resnet152 --fp8" "--model gpt2_small" "--model gpt2_small --fp8"; do
  timeout -k 10 300 python -u bench.py $M --steps 20 --no-ddp-rehearsal > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  echo "[$M] $(grep -o '"value": [0-9.]*' $O/run.log)"
done
echo done
