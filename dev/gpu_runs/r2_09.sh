#!/bin/bash
# pp engine after the SALU diet: correctness + perf table + ablations
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_09
mkdir -p $O
timeout -k 10 400 python -u tools/pp_check.py > $O/pp.log 2>&1 || exit $?
for cfg in "8192 8192 4096 --bn 256" "8192 768 3072 --bn 96"; do
  for ab in 0 1 6 7; do
    echo "ablate=$ab $cfg" >> $O/abl.log
    PDNN_PP_ABLATE=$ab timeout -k 10 60 python -u tools/pp_one.py $cfg --trace >> $O/abl.log 2>&1 || exit $?
  done
done
