#!/bin/bash
# pp engine ablations: per-slice cost with MFMA / copies / LDS reads removed
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_07
mkdir -p $O
for cfg in "8192 8192 4096 --bn 256" "8192 768 3072 --bn 96" "8192 768 3072 --bn 128" "8192 2304 3072 --bn 288"; do
  for ab in 0 1 2 3; do
    echo "ablate=$ab" >> $O/abl.log
    PDNN_PP_ABLATE=$ab timeout -k 10 60 python -u tools/pp_one.py $cfg --trace >> $O/abl.log 2>&1 || exit $?
  done
done
