#!/bin/bash
# direct 3x3 wgrad: per-kernel split (main vs reduce) under rocprofv3
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_45
mkdir -p $O
cd /tmp
W3_ABLS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o w3 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/w3_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | tail -5
python3 - <<'PY'
import csv, collections, glob, os
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r3_45/prof/**/w3_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
PY
