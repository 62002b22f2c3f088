#!/bin/bash
# why a K = 768 ping-pong item costs ~13 us more than its slices: instruction-fetch / wait counters on the LM-head
# shape (22 items per block) vs 8192^3 (4 items per block)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_11
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o -E "\b(SQC|SQ)_[A-Z0-9_]*(ICACHE|IFETCH|INST_LEVEL|INSTS_LDS|LDS_BANK)[A-Z0-9_]*" $O/avail.txt | sort -u > $O/avail_sel.txt || true
cat $O/avail_sel.txt
P=$GRAFT_REPO_ROOT/dev/probes/pp_one.py
cd /tmp
pass() {
  local n=$1; shift
  local c="$1"; shift
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --stats -d /tmp/$n -o $n --output-format csv -- python3 $P "$@" --bn 288 --iters 5 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  find /tmp/$n -name "*counter_collection.csv" -exec cp {} $O/$n.csv \;
}
Q1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VALU"
pass head_q1 "$Q1" 8192 50304 768 && pass big_q1 "$Q1" 8192 8192 8192 || exit 1
if grep -q "SQC_ICACHE_MISSES" $O/avail_sel.txt && grep -q "SQC_ICACHE_HITS" $O/avail_sel.txt; then
  pass head_q2 "SQC_ICACHE_MISSES SQC_ICACHE_HITS" 8192 50304 768 && pass big_q2 "SQC_ICACHE_MISSES SQC_ICACHE_HITS" 8192 8192 8192 || exit 1
fi
cd $GRAFT_REPO_ROOT
python3 - <<'PY' > $O/summary.txt
import csv, glob, os, collections
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r6_11"
for f in sorted(glob.glob(O + "/*_q*.csv")):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "gemm_pp" not in r.get("Kernel_Name", ""): continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(os.path.basename(f), {k: round(v / max(n[k], 1)) for k, v in sorted(acc.items())})
PY
cat $O/summary.txt
echo done
