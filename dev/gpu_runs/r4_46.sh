#!/bin/bash
# ds_read_b64_tr_b8 lane-semantics probe; fp8 halo conv NB = 64 (784 blocks at stage 3) vs 128
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_46
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./dev/probes/tr8_probe > $O/tr8.txt 2>&1 || { cat $O/tr8.txt; exit 1; }
cat $O/tr8.txt
timeout -k 10 120 python3 dev/probes/c3_fp8.py > $O/nb128.jsonl 2>&1 || exit 1
PDNN_F8NB=64 timeout -k 10 120 python3 dev/probes/c3_fp8.py > $O/nb64.jsonl 2>&1 || exit 1
cat $O/nb128.jsonl $O/nb64.jsonl
