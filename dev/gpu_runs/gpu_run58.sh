#!/bin/bash
# glds engine grid-size threshold A/B (PDNN_GLDS_MIN_TILES) on the ResNet-50 step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run58
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for rep in 1 2; do for th in 64 128 160 192; do
  PDNN_GLDS_MIN_TILES=$th $T 200 python bench.py > $O/bench_t${th}_$rep.log 2>&1 || exit $?
done; done
