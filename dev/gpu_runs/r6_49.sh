#!/bin/bash
# cross-entropy training forward that writes the unscaled gradient (tuning xent_fused): tests + GPT-2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_49
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k xent tests/test_transformer_gpu.py tests/test_graphs_gpu.py tests/test_trajectory_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
run x0_$i PDNN_TUNE=xent_fused=0 || exit 1
run x1_$i || exit 1
done
echo done
