#!/bin/bash
# end-of-round-4 ResNet-50 PMC roofline (3 passes) + per-grid kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_41
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --graph off --no-ddp-rehearsal"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d /tmp/q1 -o q1 --output-format csv -- python3 $B > $O/q1.log 2>&1 || exit $?
find /tmp/q1 -name "*counter_collection.csv" -exec cp {} $O/q1_counters.csv \;
find /tmp/q1 -name "*kernel_trace.csv" -exec cp {} $O/q1_trace.csv \;
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d /tmp/q2 -o q2 --output-format csv -- python3 $B > $O/q2.log 2>&1 || exit $?
find /tmp/q2 -name "*counter_collection.csv" -exec cp {} $O/q2_counters.csv \;
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d /tmp/q3 -o q3 --output-format csv -- python3 $B > $O/q3.log 2>&1 || exit $?
find /tmp/q3 -name "*counter_collection.csv" -exec cp {} $O/q3_counters.csv \;
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q4 -o q4 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-ddp-rehearsal > $O/q4.log 2>&1 || exit $?
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/q4_trace.csv \;
cd $R && python3 tools/pmc_summary.py $O --steps 3 --top 40 > $O/pmc_summary.txt 2>&1
python3 tools/prof_summary.py $O/q4_trace.csv --steps 3 --by-grid --top 80 > $O/grid_summary.txt 2>&1
head -3 $O/pmc_summary.txt; head -2 $O/grid_summary.txt
echo done
