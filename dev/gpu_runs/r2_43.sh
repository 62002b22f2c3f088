#!/bin/bash
# PDNN_LOWK_BN64 default 4: GPU suite; larger thresholds A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_43
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 8; [ $rc -le 1 ] || exit $rc
run() { n=$1; shift; e=$1; shift; env $e timeout -k 10 200 python -u bench.py --steps 30 "$@" > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run k4_$i PDNN_X=0
run k8_$i PDNN_LOWK_BN64=8
run k16_$i PDNN_LOWK_BN64=16
run kall_$i PDNN_LOWK_BN64=100000
done
run r152 PDNN_X=0 --model resnet152 --steps 10 --warmup 5 || true
echo done
