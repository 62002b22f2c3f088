#!/bin/bash
# pp engine K-scan (per-tile overhead vs per-slice cost) + hipBLASLt kernel names for the GPT-2 shapes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_15
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R/dev/probes
timeout -k 10 300 python3 pp_kscan.py > $O/kscan.jsonl 2> $O/kscan.err || { tail -20 $O/kscan.err; exit 1; }
cat $O/kscan.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d /tmp/h1 -o h1 --output-format csv -- python3 $R/dev/probes/gpt2_gemms.py > $O/h1.log 2>&1 || exit $?
find /tmp/h1 -name "*kernel_stats.csv" -exec cp {} $O/stats.csv \;
python3 -c "
import csv
for r in csv.DictReader(open('$O/stats.csv')):
    if r['Name'].startswith('Cijk'): print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:90])
"
