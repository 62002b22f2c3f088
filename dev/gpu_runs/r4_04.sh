#!/bin/bash
# host-vs-GPU timeline of the flagship step (kernel trace + HIP runtime trace: host lead per kernel, compute-stream
# gaps by cause), and the whole step as a replayed hipGraph (two-stream capture) against eager
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_04
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/q4 -o r50 --output-format csv -- python3 $R/bench.py --steps 4 --warmup 4 --graph off --no-ddp-rehearsal > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/r50_kernel_trace.csv \;
find /tmp/q4 -name "*hip_api_trace.csv" -exec cp {} $O/r50_hip_api_trace.csv \;
cd $R
python3 tools/stream_timeline.py $O/r50_kernel_trace.csv > $O/timeline.txt 2>&1; head -20 $O/timeline.txt
python3 tools/host_lead.py $O/r50 > $O/host_lead.txt 2>&1; head -30 $O/host_lead.txt
python3 tools/prof_summary.py $O/r50_kernel_trace.csv --steps 3 --top 40 > $O/summary.txt 2>&1
timeout -k 10 300 python -u bench.py --graph on --no-ddp-rehearsal > $O/bench_graph.log 2>&1 || { tail -20 $O/bench_graph.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench_graph.log
echo done
