#!/bin/bash
# engine-selection knobs re-swept with the 128x64 short-reduction tiles (PDNN_LOWK_BN64=24 default)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_46
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run base$i PDNN_X=0
run fwdk1200_$i PDNN_GLDS_FWD_K=1200
run fwdknever_$i PDNN_GLDS_FWD_K=100000
run ppdgradk512_$i PDNN_PP_CONV_DGRAD_K=512
run ppdgradk1024_$i PDNN_PP_CONV_DGRAD_K=1024
run mintiles384_$i PDNN_GLDS_MIN_TILES=384
done
echo done
