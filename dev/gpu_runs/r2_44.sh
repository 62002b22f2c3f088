#!/bin/bash
# PDNN_LOWK_BN64 default 16: GPU suite; neighbouring thresholds A/B, GPT-2 check
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_44
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 8; [ $rc -le 1 ] || exit $rc
run() { n=$1; shift; e=$1; shift; env $e timeout -k 10 200 python -u bench.py --steps 30 "$@" > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run k16_$i PDNN_X=0
run k12_$i PDNN_LOWK_BN64=12
run k24_$i PDNN_LOWK_BN64=24
run k36_$i PDNN_LOWK_BN64=36
done
run r152 PDNN_X=0 --model resnet152 --steps 10 --warmup 5
run gpt2 PDNN_X=0 --model gpt2_small --warmup 5
echo done
