#!/bin/bash
# attention backward: delta formed inside the dQ kernel (default) vs a separate delta launch, with the wide kernels
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_67
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs --no-plain-run > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2 3; do
run d1_$i PDNN_TUNE=attn_delta_in_dq=1 || exit 1
run d0_$i PDNN_TUNE=attn_delta_in_dq=0 || exit 1
done
echo done
