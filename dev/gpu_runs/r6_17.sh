#!/bin/bash
# ResNet-50 routing A/B after the ping-pong epilogue changes: BN-backward 1x1 dgrads from K = 512 on pp, halo 3x3 at 7x7,
# stride-2 halo forward everywhere
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_17
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run base$i PDNN_TUNE=pp_conv_fwd_c=512 && run bnk$i PDNN_TUNE=pp_dgrad_bn_k=512 && run c3f$i PDNN_TUNE=conv3x3_force=1 && run s2f$i PDNN_TUNE=s2_halo=35 || exit 1
done
echo done
