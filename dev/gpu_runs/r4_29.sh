#!/bin/bash
# PMC of the stride-2 data gradients (128-row implicit-GEMM engine, conv-transposed gather): VALU vs MFMA vs waits
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_29
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM -d /tmp/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/dev/probes/strided_dgrad.py > $O/p1.log 2>&1 || exit $?
find /tmp/p1 -name "*counter_collection.csv" -exec cp {} $O/p1_counters.csv \;
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY -d /tmp/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/dev/probes/strided_dgrad.py > $O/p2.log 2>&1 || exit $?
find /tmp/p2 -name "*counter_collection.csv" -exec cp {} $O/p2_counters.csv \;
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv, collections, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r4_29"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in ("p1_counters.csv", "p2_counters.csv"):
    for r in csv.DictReader(open(f"{O}/{f}")):
        n = r["Kernel_Name"][:60]
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, d in agg.items():
    if "gemm" in n:
        print(n, {k: f"{v:.3g}" for k, v in sorted(d.items())})
PY
