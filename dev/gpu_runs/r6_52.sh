#!/bin/bash
# GPT-2 DDP path at N = 1: split tied embedding (default) vs one dense tied bucket (PDNN_DDP_SPLIT_TIED=0)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_52
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
run s1_$i || exit 1
run s0_$i PDNN_DDP_SPLIT_TIED=0 || exit 1
done
echo done
