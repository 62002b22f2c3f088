#!/bin/bash
# GPT-2 N = 1 DDP bucket size re-measured after the round's changes: 256 MB (default) vs 512 / 128
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_57
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs --no-plain-run "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run b256_$i || exit 1
run b512_$i --bucket-mb 512 || exit 1
run b128_$i --bucket-mb 128 || exit 1
done
echo done
