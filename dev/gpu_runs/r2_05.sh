#!/bin/bash
# pp engine phase traces (where does the time of a short-K GEMM go) + K sweep
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_05
mkdir -p $O
for cfg in "8192 2304 768 --bn 288" "8192 2304 1536 --bn 288" "8192 2304 3072 --bn 288" "8192 50304 768 --bn 256" "8192 768 3072 --bn 128" "8192 768 3072 --bn 96" "8192 3072 768 --bn 192" "8192 8192 8192 --bn 256" "8192 8192 1024 --bn 256"; do
  timeout -k 10 60 python -u tools/pp_one.py $cfg --trace >> $O/trace.log 2>&1 || exit $?
done
