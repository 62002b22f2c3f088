#!/bin/bash
# attn_bwd_wide 1 vs 3 (dK / dV with 32 keys per wave too), three same-box pairs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_62
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs --no-plain-run > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2 3; do
run w1_$i PDNN_TUNE=attn_bwd_wide=1 || exit 1
run w3_$i PDNN_TUNE=attn_bwd_wide=3 || exit 1
done
echo done
