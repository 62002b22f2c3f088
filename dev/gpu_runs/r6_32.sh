#!/bin/bash
# stage-1 conv3: a2 folded (weight gradient with the operand prologue on the implicit-GEMM engine, 5% of peak) vs
# a2 materialised with the stage-1 1x1 weight gradients on the ping-pong engine
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_32
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2 3; do
run base_$i PDNN_TUNE=a2_fold=1 && run nofold_pp_$i PDNN_TUNE=a2_fold=0,wgrad1x1_pp_pix=802816 && run nofold_$i PDNN_TUNE=a2_fold=0 || exit 1
done
echo done
