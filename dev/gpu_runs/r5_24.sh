#!/bin/bash
# ResNet-50 A/B: conv3 K = 512 data gradients (stage 2) on the ping-pong engine with 64-deep slices (pp_dgrad_bn_k=512)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_24
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/base_$i.json 2> $O/base_$i.err || { tail -20 $O/base_$i.err; exit 1; }
  PDNN_TUNE=pp_dgrad_bn_k=512 timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/k512_$i.json 2> $O/k512_$i.err || { tail -20 $O/k512_$i.err; exit 1; }
  for v in base k512; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'])"; done
done
echo done
