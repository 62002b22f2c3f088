#!/bin/bash
# ResNet-50: long-reduction 1x1 weight-gradient splits planned for fewer CUs (wgrad_long_cus), same box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_42
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 - > $O/plans.txt 2>&1 <<'PY' || { cat $O/plans.txt; exit 1; }
from pytorch_distributed_nn_amd.ops import kernels as K
for cus in (0, 192, 128, 64):
    K.tune_set("wgrad_long_cus", cus)
    row = []
    for (Ko, C, P) in ((128, 512, 200704), (512, 128, 200704), (256, 1024, 50176), (1024, 256, 50176), (512, 2048, 12544), (2048, 512, 12544), (256, 512, 50176)):
        row.append(f"{Ko}x{C}x{P}:{K.lib().pdnn_pp_wgrad_splits_long(Ko, C, P)}")
    print(cus, " ".join(row))
PY
cat $O/plans.txt
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
for c in 0 192 128; do
run c${c}_$i PDNN_TUNE=wgrad_long_cus=$c || exit 1
done
done
echo done
