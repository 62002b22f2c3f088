#!/bin/bash
# per-item cost model of the ping-pong engine on the LM-head shape: K sweep (item time = overhead + K x rate)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_10
mkdir -p $O
cd $GRAFT_REPO_ROOT
P=dev/probes/pp_one.py
for bn in 288 256; do for k in 768 1536 3072 6144; do
  PDNN_TUNE=pp_epi_slack=1 timeout -k 10 60 python3 $P 8192 50304 $k --bn $bn --trace 2>&1 | grep -v amdgpu.ids | tee -a $O/ksweep.txt || exit 1
done; done
PDNN_TUNE=pp_epi_slack=1 timeout -k 10 60 python3 $P 8192 8192 8192 --bn 256 --trace 2>&1 | grep -v amdgpu.ids | tee -a $O/ksweep.txt || exit 1
echo done
