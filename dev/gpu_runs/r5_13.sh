#!/bin/bash
# pp engine uneven K-splits (GPT-2 weight gradients fill 216-252 CUs instead of 144): tests, A/B, breakdown
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_13
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad or gpt2 or colsum or transpose" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/old_$i.json 2> $O/old_$i.err) || { tail -20 $O/old_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  for v in old new; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'])"; done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g6 -o g6 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g6.log 2>&1 || exit $?
find /tmp/g6 -name "*kernel_trace.csv" -exec cp {} $O/g6_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g6_trace.csv --steps 3 --by-grid --top 50 > $O/grid_summary.txt 2>&1
head -16 $O/grid_summary.txt
echo done
