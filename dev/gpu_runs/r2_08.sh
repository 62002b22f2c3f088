#!/bin/bash
# pp engine: ablation bitmask sweep + 160 KiB ring variant
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_08
mkdir -p $O
for cfg in "8192 8192 4096 --bn 256" "8192 768 3072 --bn 96"; do
  for ab in 0 1 2 3 4 5 6 7; do
    echo "ablate=$ab $cfg" >> $O/abl.log
    PDNN_PP_ABLATE=$ab timeout -k 10 60 python -u tools/pp_one.py $cfg --trace >> $O/abl.log 2>&1 || exit $?
  done
done
for cfg in "8192 8192 4096 --bn 257" "8192 8192 4096 --bn 256" "8192 50304 768 --bn 257" "8192 50304 768 --bn 256"; do
  timeout -k 10 60 python -u tools/pp_one.py $cfg --trace >> $O/ring.log 2>&1 || exit $?
done
