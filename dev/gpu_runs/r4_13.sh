#!/bin/bash
# per-epilogue cost of the ping-pong GEMM on the GPT-2 shapes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_13
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u dev/probes/epi_cost.py > $O/epi.log 2>&1 || { tail -20 $O/epi.log; exit 1; }
grep shape $O/epi.log
