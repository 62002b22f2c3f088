#!/bin/bash
# GPT-2 bias gradients fused into the weight-gradient GEMMs (row sums against a ones fragment): numerics + A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_21
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -q --timeout 300 --timeout-method thread -k "wgrad or gpt2 or colsum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=bias_in_wgrad=0 timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/off_$i.json 2> $O/off_$i.err || { tail -20 $O/off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g7 -o g7 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g7.log 2>&1 || exit $?
find /tmp/g7 -name "*kernel_trace.csv" -exec cp {} $O/g7_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g7_trace.csv --steps 3 --by-grid --top 50 > $O/grid_summary.txt 2>&1
head -30 $O/grid_summary.txt
echo done
