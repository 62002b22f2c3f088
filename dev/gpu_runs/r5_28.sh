#!/bin/bash
# GPT-2: per-block batched transposed-weight refresh (one launch per block backward) vs per-weight lazy transposes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_28
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 170 --timeout-method thread -k "gpt2" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=wt_layer_batch=0 timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/off_$i.json 2> $O/off_$i.err || { tail -20 $O/off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
echo done
