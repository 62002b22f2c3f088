#!/bin/bash
# driver-shaped N=1 bench (headline + plain child + configs 4/5 children, wall time) and the round-6 PMC byte ledger
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_07
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k "dgrad" > $O/flip_tests.log 2>&1 || { tail -30 $O/flip_tests.log; exit 1; }
tail -1 $O/flip_tests.log
S=$(date +%s)
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bench wall s: $(( $(date +%s) - S ))"
python3 -c "
import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu'])
for k,v in (d.get('extra_configs') or {}).items(): print(k, v.get('value'), v.get('ms_per_step'), v.get('wall_s'), v.get('error'))"
B="$GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --plain"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d /tmp/q1 -o q1 --output-format csv -- python3 $B > $O/q1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d /tmp/q2 -o q2 --output-format csv -- python3 $B > $O/q2.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d /tmp/q3 -o q3 --output-format csv -- python3 $B > $O/q3.log 2>&1 || exit $?
for q in q1 q2 q3; do find /tmp/$q -name "*counter_collection.csv" -exec cp {} $O/${q}_counters.csv \; ; done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py $O --steps 6 --top 70 --ledger > $O/pmc_summary.txt 2>&1
head -4 $O/pmc_summary.txt
tail -14 $O/pmc_summary.txt
echo done
