#!/bin/bash
# GPT-2 weight gradients on the side stream (gpt2_side_wgrad): numerics test + A/B; new split-K test
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_33
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "splitk" > $O/tests0.log 2>&1 || { tail -40 $O/tests0.log; exit 1; }
tail -1 $O/tests0.log
PDNN_TUNE=gpt2_side_wgrad=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_trajectory_gpu.py tests/test_ddp_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d.get('final_loss'))"
}
for i in 1 2; do
run g0_$i PDNN_TUNE=gpt2_side_wgrad=0 && run g1_$i PDNN_TUNE=gpt2_side_wgrad=1 || exit 1
done
echo done
