#!/bin/bash
# env-only knobs under the final defaults
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_49
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run base$i PDNN_X=0
run nostage$i PDNN_STAGED_STORE=0
run noglds$i PDNN_GLDS=0
run ppbnb$i PDNN_PP_CONV_BNB=1
run s1024_$i PDNN_SPLIT_BLOCKS=1024
done
echo done
