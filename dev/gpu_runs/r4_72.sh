#!/bin/bash
# BN reduce grids 512 blocks / 32 rows on top of the 512-block streaming grids: full GPU suite + smoke, driver-style bench x2, GPT-2,
# ResNet-152 bf16/fp8 pair, and a kernel trace for the per-grid breakdown
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_72
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 400 python3 bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  cut -c1-160 $O/bench_$i.json
done
timeout -k 10 400 python3 bench.py --model gpt2 > $O/gpt2.json 2> $O/gpt2.err || { tail -20 $O/gpt2.err; exit 1; }
cut -c1-160 $O/gpt2.json
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-110 $O/bf16_*.json $O/fp8_*.json
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q4 -o q4 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-ddp-rehearsal > $O/q4.log 2>&1 || exit $?
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/q4_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/q4_trace.csv --steps 3 --by-grid --top 80 > $O/grid_summary.txt 2>&1
python3 tools/prof_summary.py $O/q4_trace.csv --steps 3 --top 60 > $O/summary.txt 2>&1
head -3 $O/grid_summary.txt
echo done
