#!/bin/bash
# split-K block target of the weight gradients (side stream) A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_48
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run base$i PDNN_X=0
run s256_$i PDNN_SPLIT_BLOCKS=256
run s384_$i PDNN_SPLIT_BLOCKS=384
run s768_$i PDNN_SPLIT_BLOCKS=768
done
echo done
