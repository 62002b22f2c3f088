#!/bin/bash
# --opt-overlap (per-bucket optimizer updates during the backward) re-measured with the side-stream weight gradients
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_48
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-extra-configs --no-plain-run "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run g0_$i --model gpt2_small || exit 1
run g1_$i --model gpt2_small --opt-overlap || exit 1
run r0_$i || exit 1
run r1_$i --opt-overlap || exit 1
done
echo done
