#!/bin/bash
# GPT-2: batched side-stream transposes at forward start + one-launch atomic bias-gradient colsum; A/B vs HEAD
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_09
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "transformer or gpt2 or colsum or transpose or flash or attention or layernorm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/old_$i.json 2> $O/old_$i.err) || { tail -20 $O/old_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  for v in old new; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'])"; done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g5 -o g5 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g5.log 2>&1 || exit $?
find /tmp/g5 -name "*kernel_trace.csv" -exec cp {} $O/g5_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g5_trace.csv --steps 3 --by-grid --top 50 > $O/grid_summary.txt 2>&1
head -30 $O/grid_summary.txt
echo done
