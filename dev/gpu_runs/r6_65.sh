#!/bin/bash
# ResNet-50: 1x1 forwards on the ping-pong engine from C >= 256 (pp_conv_fwd_c 256) vs 512 (default), same box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_65
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-extra-configs --no-plain-run > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2 3; do
run c512_$i PDNN_TUNE=pp_conv_fwd_c=512 || exit 1
run c256_$i PDNN_TUNE=pp_conv_fwd_c=256 || exit 1
done
echo done
