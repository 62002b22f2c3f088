#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run37
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d /tmp/p1 -o p1 --output-format csv -- python3 $R/tools/attn_once.py 1 > $O/p1.log 2>&1 || exit $?
cp /tmp/p1/p1_counter_collection.csv $O/ 2>/dev/null || find /tmp/p1 -name "*.csv" -exec cp {} $O/ \;
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY -d /tmp/p2 -o p2 --output-format csv -- python3 $R/tools/attn_once.py 1 > $O/p2.log 2>&1 || exit $?
find /tmp/p2 -name "*counter*.csv" -exec cp {} $O/p2_counters.csv \;
ls /tmp/p1 /tmp/p2 > $O/ls.txt
