#!/bin/bash
# AdamW overlapped with the backward (GPT-2, one GPU): test + A/B vs graphed / eager whole-arena step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_41
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_overlap_gpu.py tests/test_transformer_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
run() { n=$1; shift; e=$1; shift; env $e timeout -k 10 200 python -u bench.py --model gpt2_small --steps 30 --warmup 5 "$@" > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-120)" || exit 1; }
for i in 1 2; do
run graph$i PDNN_X=0
run eager$i PDNN_X=0 --graph off
run overlap$i PDNN_OPT_OVERLAP=1
done
echo done
