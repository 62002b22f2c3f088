#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run23
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
C2="SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL GRBM_GUI_ACTIVE"
C3="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"
for who in ours torch; do
  i=0
  for C in "$C1" "$C2" "$C3"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d /tmp/p_${who}_$i -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/exp_pmc.py 802816 256 64 $who > $O/log_${who}_$i.txt 2>&1 || exit $?
    python3 - "$who" "$i" <<'PY' >> $O/pmc_summary.txt
import csv, sys, collections, glob
who, i = sys.argv[1], sys.argv[2]
f = glob.glob(f"/tmp/p_{who}_{i}/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    if "gemm" in k.lower() or "Cijk" in k:
        print(who, i, k, {a: "%.4g" % (b / max(cnt[(k, a)], 1)) for a, b in v.items()})
PY
  done
done
