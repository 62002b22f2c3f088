#!/bin/bash
# end-of-round-6 ResNet-50 PMC ledger (same 3 passes as r6_07 / r5_52) + the GPT-2 kernel breakdown
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_31
mkdir -p $O
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 3 --warmup 3 --plain"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d /tmp/q1 -o q1 --output-format csv -- python3 $B > $O/q1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d /tmp/q2 -o q2 --output-format csv -- python3 $B > $O/q2.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d /tmp/q3 -o q3 --output-format csv -- python3 $B > $O/q3.log 2>&1 || exit $?
for q in q1 q2 q3; do find /tmp/$q -name "*counter_collection.csv" -exec cp {} $O/${q}_counters.csv \; ; done
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g31 -o g31 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 5 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/g31.log 2>&1 || exit $?
find /tmp/g31 -name "*kernel_trace.csv" -exec cp {} $O/g31_trace.csv \;
cd $R && python3 tools/pmc_summary.py $O --steps 6 --top 70 --ledger > $O/pmc_summary.txt 2>&1
python3 tools/prof_summary.py $O/g31_trace.csv --steps 3 --by-grid --top 40 > $O/gpt2_grid_summary.txt 2>&1
head -4 $O/pmc_summary.txt
tail -14 $O/pmc_summary.txt
head -3 $O/gpt2_grid_summary.txt
echo done
