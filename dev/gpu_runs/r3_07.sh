#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_07
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 30 > $O/bench_m1_$i.log 2>&1 && tail -n 1 $O/bench_m1_$i.log | cut -c1-120 || exit 1
PDNN_MASKED_RES=0 timeout -k 10 200 python -u bench.py --steps 30 > $O/bench_m0_$i.log 2>&1 && tail -n 1 $O/bench_m0_$i.log | cut -c1-120 || exit 1
done
PDNN_CONV3X3=0 timeout -k 10 200 python -u bench.py --steps 30 > $O/bench_c3off.log 2>&1 && tail -n 1 $O/bench_c3off.log | cut -c1-120 || exit 1
echo done
