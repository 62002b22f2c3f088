#!/bin/bash
# follow-up of run62: data gradient off the glds engine (+2.3%), combined with forward cut-offs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run63
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
run() {  # tag env...
  local tag=$1; shift
  env "$@" $T 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_${tag}_$rep.log 2>&1
}
D="PDNN_GLDS_DGRAD_N=100000 PDNN_GLDS_DGRAD_K=100000"
for rep in 1 2; do
  run dgnever $D || exit $?
  run dgnever_fwk1024 $D PDNN_GLDS_FWD_K=1024 || exit $?
  run dgnever_fwk2048 $D PDNN_GLDS_FWD_K=2048 || exit $?
  run dgnever_fwnever $D PDNN_GLDS_FWD_K=100000 || exit $?
  run dgk2048 PDNN_GLDS_DGRAD_N=100000 PDNN_GLDS_DGRAD_K=2048 || exit $?
  run allreg PDNN_GLDS=0 || exit $?
done
