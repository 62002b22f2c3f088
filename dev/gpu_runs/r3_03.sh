#!/bin/bash
# 1x1 conv engine A/B at the ResNet-50 bottleneck shapes (fused prologue vs materialised a2; pp on/off)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_03
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/default.log 2>&1 && cat $O/default.log || exit 1
PDNN_PP_CONV_FWD_K=0 PDNN_PP_CONV_BNB=1 PDNN_PP_CONV_DGRAD_K=0 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/pp_all.log 2>&1 && cat $O/pp_all.log || exit 1
PDNN_GLDS=2 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/glds.log 2>&1 && cat $O/glds.log || exit 1
PDNN_LOWK_BN64=0 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/bn128.log 2>&1 && cat $O/bn128.log || exit 1
echo done
