#!/bin/bash
# persistent pp engine: correctness + perf table, then PMC passes on three configurations
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_04
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/pp_check.py > $O/pp.log 2>&1 || exit $?
cd /tmp
for cfg in "8192 8192 8192 --bn 256" "8192 768 3072 --bn 96" "8192 768 3072 --bn 128" "8192 2304 768 --bn 288" "8192 50304 768 --bn 256"; do
  tag=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE -d /tmp/p1_$tag -o p1 --output-format csv -- python3 $R/tools/pp_one.py $cfg --iters 5 > $O/p1_$tag.log 2>&1 || exit $?
  find /tmp/p1_$tag -name "*counter_collection.csv" -exec cp {} $O/p1_$tag.csv \;
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM -d /tmp/p2_$tag -o p2 --output-format csv -- python3 $R/tools/pp_one.py $cfg --iters 5 > $O/p2_$tag.log 2>&1 || exit $?
  find /tmp/p2_$tag -name "*counter_collection.csv" -exec cp {} $O/p2_$tag.csv \;
done
