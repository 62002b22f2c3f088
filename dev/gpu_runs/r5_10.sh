#!/bin/bash
# GPT-2 A/B: HEAD vs transposes-at-forward-start (main / side stream / off) x atomic colsum on/off
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_10
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/old_$i.json 2> $O/old_$i.err) || { tail -20 $O/old_$i.err; exit 1; }
  for v in "wt_prefetch=1" "wt_prefetch=2" "wt_prefetch=0" "wt_prefetch=1,colsum_atomic=0"; do
    n=$(echo $v | tr '=,' '__')
    PDNN_TUNE=$v timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -20 $O/${n}_$i.err; exit 1; }
  done
  for f in $O/*_$i.json; do python3 -c "import json;d=json.load(open('$f'));print('$(basename $f)',d['value'],d['ms_per_step'])"; done
done
echo done
