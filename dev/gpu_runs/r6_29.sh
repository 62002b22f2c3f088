#!/bin/bash
# stem max-pool backward + BN reduce: 2 vs 3 blocks per CU (168-VGPR cap): tests, isolation, ResNet-50 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_29
mkdir -p $O
cd $GRAFT_REPO_ROOT
PDNN_TUNE=maxpool_bwd_per_cu=3 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py tests/test_kernels_gpu.py -k "pool or stem" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for b in 2 3; do
PDNN_TUNE=maxpool_bwd_per_cu=$b timeout -k 10 200 python3 dev/probes/stem_bwd_cost.py > $O/stem_$b.json 2> $O/stem_$b.err || { tail -20 $O/stem_$b.err; exit 1; }
echo "per_cu $b $(python3 -c "import json;d=json.load(open('$O/stem_$b.json'));print(d['maxpool_bwd_bnred_us'])")"
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run m2_$i PDNN_TUNE=maxpool_bwd_per_cu=2 && run m3_$i PDNN_TUNE=maxpool_bwd_per_cu=3 || exit 1
done
echo done
