#!/bin/bash
# GPT-2 linear weight-gradient plan sized for the side stream (tuning wgrad_plan_cus): plans, tests, same-box A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_40
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 - > $O/plans.txt 2>&1 <<'PY' || { cat $O/plans.txt; exit 1; }
from pytorch_distributed_nn_amd.ops import kernels as K
for cus in (0, 192, 128, 96, 64):
    K.tune_set("wgrad_plan_cus", cus)
    row = []
    for nm, M, N in (("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072)):
        bn, s = divmod(K.lib().pdnn_pp_wgrad_plan(M, N, 8192), 1000)
        row.append(f"{nm} {bn}x{s}")
    print(cus, " | ".join(row))
PY
cat $O/plans.txt
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tuning_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
run c0_$i || exit 1
run c128_$i PDNN_TUNE=wgrad_plan_cus=128 || exit 1
run c64_$i PDNN_TUNE=wgrad_plan_cus=64 || exit 1
done
echo done
