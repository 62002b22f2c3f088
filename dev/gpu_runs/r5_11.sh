#!/bin/bash
# GPT-2 host issue time vs GPU time (DDP path), cProfile
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_11
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
PDNN_TUNE=wt_prefetch=0 timeout -k 10 300 python3 dev/probes/gpt2_host.py > $O/host.txt 2>&1 || { tail -20 $O/host.txt; exit 1; }
head -60 $O/host.txt
