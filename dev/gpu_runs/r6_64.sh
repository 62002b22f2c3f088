#!/bin/bash
# ping-pong tile width planned for fewer free CUs (tuning pp_plan_cus: the side stream holds CUs during the
# backward): widths chosen, tuning test, GPT-2 / ResNet-50 same-box A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_64
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tuning_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-extra-configs --no-plain-run $EXTRA > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
EXTRA="--model gpt2_small" run g0_$i PDNN_TUNE=pp_plan_cus=0 || exit 1
EXTRA="--model gpt2_small" run g160_$i PDNN_TUNE=pp_plan_cus=160 || exit 1
EXTRA="--model gpt2_small" run g192_$i PDNN_TUNE=pp_plan_cus=192 || exit 1
EXTRA="" run r0_$i PDNN_TUNE=pp_plan_cus=0 || exit 1
EXTRA="" run r160_$i PDNN_TUNE=pp_plan_cus=160 || exit 1
done
echo done
