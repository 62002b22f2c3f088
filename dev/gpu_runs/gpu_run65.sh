#!/bin/bash
# re-sweep of the register-kernel knobs now that the data gradient runs on it (run64 defaults)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run65
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
run() {  # tag env...
  local tag=$1; shift
  env "$@" $T 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_${tag}_$rep.log 2>&1
}
for rep in 1 2; do
  run base PDNN_X=0 || exit $?
  run lowk PDNN_LOWK_BN64=1 || exit $?
  run nostage PDNN_STAGED_STORE=0 || exit $?
  run mt128 PDNN_GLDS_MIN_TILES=128 || exit $?
  run mt320 PDNN_GLDS_MIN_TILES=320 || exit $?
done
