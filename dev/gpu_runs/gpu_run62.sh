#!/bin/bash
# glds engine shape-threshold A/B on the ResNet-50 step: data-gradient (PDNN_GLDS_DGRAD_N/K) and forward
# (PDNN_GLDS_FWD_K) cut-offs between the glds 256-row engine and the register-staged 128-tile kernel
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run62
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
run() {  # tag env...
  local tag=$1; shift
  env "$@" $T 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_${tag}_$rep.log 2>&1
}
for rep in 1 2; do
  run base PDNN_X=0 || exit $?
  run dgnever PDNN_GLDS_DGRAD_N=100000 PDNN_GLDS_DGRAD_K=100000 || exit $?
  run dgn256 PDNN_GLDS_DGRAD_N=256 || exit $?
  run dgn512 PDNN_GLDS_DGRAD_N=512 PDNN_GLDS_DGRAD_K=100000 || exit $?
  run dgall PDNN_GLDS_DGRAD_N=0 || exit $?
  run fwk256 PDNN_GLDS_FWD_K=256 || exit $?
  run fwk1024 PDNN_GLDS_FWD_K=1024 || exit $?
done
