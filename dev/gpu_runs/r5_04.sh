#!/bin/bash
# BN statistics into 64 atomic bins + one-block-per-column finalize that re-zeroes them: full GPU suite, bench x2,
# kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_04
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 400 python3 bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));r=d['plain_step_1gpu'];print(d['value'],r.get('value'),r.get('error'))"
done
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q4 -o q4 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-plain-run > $O/q4.log 2>&1 || exit $?
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/q4_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/q4_trace.csv --steps 3 --by-grid --top 80 > $O/grid_summary.txt 2>&1
python3 tools/stream_timeline.py $O/q4_trace.csv > $O/timeline.txt 2>&1
head -3 $O/grid_summary.txt
echo done
