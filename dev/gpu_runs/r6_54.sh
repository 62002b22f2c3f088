#!/bin/bash
# side-stream weight-gradient plan scoped to the side stream (the tied LM head's compute-stream weight gradient plans
# for the whole chip again): tests + GPT-2 A/B vs HEAD lib/package snapshot
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_54
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tuning_gpu.py tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 60 python3 -c "
from pytorch_distributed_nn_amd.ops import kernels as K
for c in (0, 128): print('head plan cus', c, K.lib().pdnn_pp_wgrad_plan(50304, 768, 8192, c))"
run() {
  local n=$1; shift
  (cd $1 && timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err) || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
run old_$i $GRAFT_REPO_ROOT/ab_old || exit 1
run new_$i $GRAFT_REPO_ROOT || exit 1
done
echo done
