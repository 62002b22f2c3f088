#!/bin/bash
# stem kernel timing + PMC counters (instruction mix, waits)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_26
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u tools/probe_stem.py > $O/probe.log 2>&1 || { cat $O/probe.log; exit 1; }
cat $O/probe.log | tail -1
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d /tmp/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_stem.py --iters 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
find /tmp/p1 -name "*counter_collection.csv" -exec cp {} $O/p1_counters.csv \;
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD -d /tmp/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_stem.py --iters 3 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
find /tmp/p2 -name "*counter_collection.csv" -exec cp {} $O/p2_counters.csv \;
echo done
