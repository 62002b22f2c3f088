#!/bin/bash
# 128x64 tile for short reductions (PDNN_LOWK_BN64=k K-steps): A/B, plus GEMM/conv tests under the knob
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_42
mkdir -p $O
cd $GRAFT_REPO_ROOT
PDNN_LOWK_BN64=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run base$i PDNN_X=0
run k1_$i PDNN_LOWK_BN64=1
run k2_$i PDNN_LOWK_BN64=2
run k4_$i PDNN_LOWK_BN64=4
done
echo done
