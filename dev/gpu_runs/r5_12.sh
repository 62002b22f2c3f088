#!/bin/bash
# N = 768 GEMMs: ours vs hipBLASLt kernel names / times, and SQ counter pass
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_12
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp

timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d /tmp/n1 -o n1 --output-format csv -- python3 $R/dev/probes/n768_gemm.py > $O/n1.log 2>&1 || exit $?
find /tmp/n1 -name "*kernel_stats.csv" -exec cp {} $O/stats.csv \;
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_MFMA -d /tmp/n2 -o n2 --output-format csv -- python3 $R/dev/probes/n768_gemm.py > $O/n2.log 2>&1 || exit $?
find /tmp/n2 -name "*counter_collection.csv" -exec cp {} $O/pmc1.csv \;
cut -c1-250 $O/stats.csv
echo done
