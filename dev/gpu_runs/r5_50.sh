#!/bin/bash
# attention backward: delta formed inside the dQ kernel (no delta launch): tests + bench_attn + GPT-2 A/B (PDNN_TUNE)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_50
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_transformer_gpu.py tests/test_tuning_gpu.py -x -v --timeout 170 --timeout-method thread -k "attention or attn or gpt2 or delta" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PDNN_TUNE=attn_delta_in_dq=0 timeout -k 10 600 python3 -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 170 --timeout-method thread -k "attention" > $O/tests_off.log 2>&1 || { tail -40 $O/tests_off.log; exit 1; }
tail -1 $O/tests_off.log
timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_new.jsonl 2>&1 || exit 1
PDNN_TUNE=attn_delta_in_dq=0 timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_off.jsonl 2>&1 || exit 1
head -1 $O/attn_new.jsonl; head -1 $O/attn_off.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=attn_delta_in_dq=0 timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/off_$i.json 2> $O/off_$i.err || { tail -20 $O/off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
echo done
