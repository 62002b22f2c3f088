#!/bin/bash
# stage-1 1x1 weight gradients on the ping-pong engine (wgrad1x1_pp_pix 802816) after the epilogue changes: A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_30
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2 3; do
run base_$i PDNN_TUNE=wgrad1x1_pp_pix=200704 && run pp_$i PDNN_TUNE=wgrad1x1_pp_pix=802816 || exit 1
done
echo done
