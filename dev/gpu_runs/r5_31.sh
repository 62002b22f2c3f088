#!/bin/bash
# GPT-2 LM-head GEMMs (M 8192, V 50304, C 768) in isolation: in-tree pp per tile width + phase trace vs hipBLASLt
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_31
mkdir -p $O
cd $GRAFT_REPO_ROOT
P=dev/probes/pp_one.py
timeout -k 10 120 python3 dev/probes/head_torch.py 2>&1 | tee $O/torch.txt || exit 1
for bn in 0 192 256 288; do timeout -k 10 60 python3 $P 8192 50304 768 --bn $bn --trace 2>&1 | tee -a $O/fwd.txt || exit 1; done
for bn in 0 96 128 256; do timeout -k 10 60 python3 $P 8192 768 50304 --kind nn --bn $bn --trace 2>&1 | tee -a $O/dgrad.txt || exit 1; done
for bn in 0 96 128 256; do timeout -k 10 60 python3 $P 50304 768 8192 --kind wgrad --bn $bn --trace 2>&1 | tee -a $O/wgrad.txt || exit 1; done
echo done
