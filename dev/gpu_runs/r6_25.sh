#!/bin/bash
# stem weight-gradient grid (2 / 4 / 8 blocks per CU): tests, isolation, ResNet-50 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_25
mkdir -p $O
cd $GRAFT_REPO_ROOT
PDNN_TUNE=stem_wgrad_blocks=2048 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for b in 512 1024 2048; do
PDNN_TUNE=stem_wgrad_blocks=$b timeout -k 10 200 python3 dev/probes/stem_bwd_cost.py > $O/stem_$b.json 2> $O/stem_$b.err || { tail -20 $O/stem_$b.err; exit 1; }
echo "blocks $b $(cat $O/stem_$b.json)"
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run b512_$i PDNN_TUNE=stem_wgrad_blocks=512 && run b1024_$i PDNN_TUNE=stem_wgrad_blocks=1024 && run b2048_$i PDNN_TUNE=stem_wgrad_blocks=2048 || exit 1
done
echo done
