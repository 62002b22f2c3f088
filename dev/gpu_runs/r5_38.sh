#!/bin/bash
# LM-head GEMM with cross-entropy statistics in its epilogue: tests + GPT-2 A/B (PDNN_TUNE=xent_in_gemm=0) + trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_38
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 170 --timeout-method thread -k "xent or gpt2" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  m=gpt2
  timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_new_$i.json 2> $O/${m}_new_$i.err || { tail -20 $O/${m}_new_$i.err; exit 1; }
  PDNN_TUNE=xent_in_gemm=0 timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_off_$i.json 2> $O/${m}_off_$i.err || { tail -20 $O/${m}_off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${m}_${v}_$i.json'));print('$m $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g9 -o g9 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g9.log 2>&1 || exit $?
find /tmp/g9 -name "*kernel_trace.csv" -exec cp {} $O/g9_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g9_trace.csv --steps 3 --by-grid --top 60 > $O/grid_summary.txt 2>&1
head -14 $O/grid_summary.txt
echo done
