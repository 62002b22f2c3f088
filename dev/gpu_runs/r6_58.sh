#!/bin/bash
# GPT-2 transposed-weight prefetch re-measured with the side-stream weight gradients / high-priority compute stream
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_58
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs --no-plain-run > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run p0_$i PDNN_TUNE=wt_prefetch=0 || exit 1
run p1_$i PDNN_TUNE=wt_prefetch=1 || exit 1
run p2_$i PDNN_TUNE=wt_prefetch=2 || exit 1
done
echo done
