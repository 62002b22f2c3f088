#!/bin/bash
# two-stream knobs re-checked under the final defaults
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_50
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run base$i PDNN_X=0
run nodown$i PDNN_SIDE_DOWN=0
run prio0_$i PDNN_MAIN_PRIO=0
run serial$i PDNN_SIDE_WGRAD=0
done
echo done
