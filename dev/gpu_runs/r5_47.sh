#!/bin/bash
# DDP first bucket at the full cap (no 4 KB fc.bias collective): DDP GPU tests + ResNet-50 A/B vs ab_old
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_47
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  m=resnet50
  timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_new_$i.json 2> $O/${m}_new_$i.err || { tail -20 $O/${m}_new_$i.err; exit 1; }
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_old_$i.json 2> $O/${m}_old_$i.err) || { tail -20 $O/${m}_old_$i.err; exit 1; }
  for v in new old; do python3 -c "import json;d=json.load(open('$O/${m}_${v}_$i.json'));print('$m $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
echo done
