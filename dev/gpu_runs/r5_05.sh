#!/bin/bash
# same-box A/B: previous commit (per-tile slab rows + wide finalize) vs statistics bins (+ a2 fold); clean traces
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_05
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3; do
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/old_$i.json 2> $O/old_$i.err) || { tail -20 $O/old_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=a2_fold=0 timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/nofold_$i.json 2> $O/nofold_$i.err || { tail -20 $O/nofold_$i.err; exit 1; }
  for v in old new nofold; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'])"; done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q4 -o q4 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/q4.log 2>&1 || exit $?
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/q4_trace.csv \;
cd $R/ab_old
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q5 -o q5 --output-format csv -- python3 $R/ab_old/bench.py --steps 5 --warmup 3 --diag-steps 0 > $O/q5.log 2>&1 || exit $?
find /tmp/q5 -name "*kernel_trace.csv" -exec cp {} $O/q5_trace.csv \;
cd $R && python3 tools/stream_timeline.py $O/q4_trace.csv > $O/timeline_new.txt 2>&1
python3 tools/stream_timeline.py $O/q5_trace.csv > $O/timeline_old.txt 2>&1
head -4 $O/timeline_new.txt $O/timeline_old.txt
echo done
