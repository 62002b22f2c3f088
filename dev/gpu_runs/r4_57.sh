#!/bin/bash
# GPT-2: transposed weights for the data gradients built on the side stream during the forward; numerics + A/B
# (temporary PDNN_AB_NO_TPREFETCH switch), graphed (default) and eager
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_57
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_gpu.py tests/test_graphs_gpu.py tests/test_models_gpu.py tests/test_fp8_gpu.py -k "gpt or graph or transformer" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  PDNN_AB_NO_TPREFETCH=1 timeout -k 10 300 python3 bench.py --model gpt2_small --steps 20 --warmup 8 --no-ddp-rehearsal > $O/a.json 2> $O/a.err || { tail -20 $O/a.err; exit 1; }
  echo "[off] $(grep -o '"value": [0-9.]*' $O/a.json)"
  timeout -k 10 300 python3 bench.py --model gpt2_small --steps 20 --warmup 8 --no-ddp-rehearsal > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "[on]  $(grep -o '"value": [0-9.]*' $O/b.json)"
done
for i in 1 2; do
  PDNN_AB_NO_TPREFETCH=1 timeout -k 10 300 python3 bench.py --model gpt2_small --steps 20 --warmup 8 --no-ddp-rehearsal --graph off > $O/a.json 2> $O/a.err || { tail -20 $O/a.err; exit 1; }
  echo "[off eager] $(grep -o '"value": [0-9.]*' $O/a.json)"
  timeout -k 10 300 python3 bench.py --model gpt2_small --steps 20 --warmup 8 --no-ddp-rehearsal --graph off > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "[on  eager] $(grep -o '"value": [0-9.]*' $O/b.json)"
done
