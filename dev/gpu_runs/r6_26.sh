#!/bin/bash
# stem weight-gradient duration inside the ResNet-50 step (kernel trace) at 512 vs 2048 blocks
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_26
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for b in 512 2048; do
PDNN_TUNE=stem_wgrad_blocks=$b timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/s$b -o s$b --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 --plain > $O/s$b.log 2>&1 || exit $?
find /tmp/s$b -name "*kernel_trace.csv" -exec cp {} $O/s$b.csv \;
done
cd $R
python3 - <<'PY'
import csv, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r6_26"
for b in (512, 2048):
    rows = list(csv.DictReader(open(f"{O}/s{b}.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for k in ("stem_wgrad_kernel", "maxpool_bwd_bnred", "sgd_kernel"):
        v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if k in r["Kernel_Name"]]
        print(b, k, [round(x, 1) for x in v])
PY
echo done
