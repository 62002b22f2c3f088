#!/bin/bash
# (new engine defaults) PMC counters over the flagship ResNet-50 bs256 step (kernel-trace + pmc only, one counter group per pass):
# pass 1 MFMA work + busy cycles + LDS conflicts, pass 2 L2->fabric read bytes, pass 3 write bytes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run66
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --graph off"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d /tmp/q1 -o q1 --output-format csv -- python3 $B > $O/q1.log 2>&1 || exit $?
find /tmp/q1 -name "*counter_collection.csv" -exec cp {} $O/q1_counters.csv \;
find /tmp/q1 -name "*kernel_trace.csv" -exec cp {} $O/q1_trace.csv \;
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d /tmp/q2 -o q2 --output-format csv -- python3 $B > $O/q2.log 2>&1 || exit $?
find /tmp/q2 -name "*counter_collection.csv" -exec cp {} $O/q2_counters.csv \;
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d /tmp/q3 -o q3 --output-format csv -- python3 $B > $O/q3.log 2>&1 || exit $?
find /tmp/q3 -name "*counter_collection.csv" -exec cp {} $O/q3_counters.csv \;
ls -la $O > $O/ls.txt
