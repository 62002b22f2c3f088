#!/bin/bash
# engine-selection knobs re-swept under the concurrent (side-stream) schedule, ResNet-50 bs256
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_39
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
run base PDNN_X=0
run dgradk1024 PDNN_GLDS_DGRAD_K=1024
run dgradk512 PDNN_GLDS_DGRAD_K=512
run dgradn256 PDNN_GLDS_DGRAD_N=256
run fwdk512 PDNN_GLDS_FWD_K=512
run fwdk256 PDNN_GLDS_FWD_K=256
run fwdknever PDNN_GLDS_FWD_K=100000
run ppdgradk128 PDNN_PP_CONV_DGRAD_K=128
run ppbnb PDNN_PP_CONV_BNB=1
run ppfwdk512 PDNN_PP_CONV_FWD_K=512
run mintiles128 PDNN_GLDS_MIN_TILES=128
run mintiles384 PDNN_GLDS_MIN_TILES=384
run base2 PDNN_X=0
echo done
