#!/bin/bash
# GPT-2 A/B on one box: LayerNorm parameter-gradient reduction on the side stream (gpt2_side_wgrad=2) vs the
# linear weight gradients only (1)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_39
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
run s1_$i PDNN_TUNE=gpt2_side_wgrad=1 || exit 1
run s2_$i PDNN_TUNE=gpt2_side_wgrad=2 || exit 1
done
echo done
