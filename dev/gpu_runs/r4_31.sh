#!/bin/bash
# instruction mix per kernel of the ResNet-50 step (which kernels are VALU-bound)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_31
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d /tmp/m1 -o m1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --graph off --no-ddp-rehearsal > $O/m1.log 2>&1 || exit $?
find /tmp/m1 -name "*counter_collection.csv" -exec cp {} $O/m1_counters.csv \;
cd $GRAFT_REPO_ROOT && python3 - > $O/mix.txt <<'PY'
import csv, collections, os, re
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r4_31"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f"{O}/m1_counters.csv")):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:70]
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[n].add(r["Dispatch_Id"])
tot = sum(d["SQ_WAVE_CYCLES"] for d in agg.values())
print(f"{'wave%':>6} {'VALU/MFMA':>9} {'SALU/MFMA':>9} {'VMEM/MFMA':>9} {'LDS/MFMA':>8} {'waitinst%':>9}  kernel")
for n, d in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:40]:
    mf = max(d["SQ_INSTS_MFMA"], 1)
    print(f"{100*d['SQ_WAVE_CYCLES']/tot:6.1f} {d['SQ_INSTS_VALU']/mf:9.1f} {d['SQ_INSTS_SALU']/mf:9.1f} {d['SQ_INSTS_VMEM']/mf:9.2f} "
          f"{d['SQ_INSTS_LDS']/mf:8.2f} {100*d['SQ_WAIT_INST_ANY']/max(d['SQ_WAVE_CYCLES'],1):9.1f}  {n}")
PY
head -30 $O/mix.txt
