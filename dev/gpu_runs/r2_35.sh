#!/bin/bash
# stream priorities (side low / main high) and the forward shortcut conv on the side stream: A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_35
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())" || exit 1
PDNN_SIDE_DOWN=1 timeout -k 10 300 python -u -m pytest tests/test_fused_blocks_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c1-120)" || exit 1; }
for i in 1 2; do
run base$i PDNN_X=0
run sidelow$i PDNN_SIDE_PRIO=1
run mainhigh$i PDNN_MAIN_PRIO=-1
run down$i PDNN_SIDE_DOWN=1
run down_mainhigh$i PDNN_SIDE_DOWN=1 PDNN_MAIN_PRIO=-1
done
echo done
