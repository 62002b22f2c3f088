#!/bin/bash
# GPT-2 N = 768 GEMMs: tile widths and split-K vs hipBLASLt
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_20
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u dev/probes/splitk_n768.py > $O/sk.log 2>&1 || { tail -20 $O/sk.log; exit 1; }
grep shape $O/sk.log
