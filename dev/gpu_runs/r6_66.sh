#!/bin/bash
# ResNet-50: BN-backward 1x1 data gradients on the ping-pong engine from K = 512 vs 1024 (default), same box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_66
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-extra-configs --no-plain-run > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2 3; do
run k1024_$i PDNN_TUNE=pp_dgrad_bn_k=1024 || exit 1
run k512_$i PDNN_TUNE=pp_dgrad_bn_k=512 || exit 1
done
echo done
