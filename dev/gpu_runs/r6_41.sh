#!/bin/bash
# GPT-2 wgrad_plan_cus finer sweep, same box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_41
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
for c in 0 160 144 128 112; do
run c${c}_$i PDNN_TUNE=wgrad_plan_cus=$c || exit 1
done
done
echo done
