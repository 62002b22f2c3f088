#!/bin/bash
# 64-deep bf16 slices for 96 / 128-wide tiles: numerics, per-GEMM timings, GPT-2 A/B (pp_sk64 = 1 vs 0)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_18
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "pp_narrow or wgrad or gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 dev/probes/gpt2_gemms.py > $O/gemms.jsonl 2> $O/gemms.err || { tail -20 $O/gemms.err; exit 1; }
cut -c1-330 $O/gemms.jsonl
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=pp_sk64=0 timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/off_$i.json 2> $O/off_$i.err || { tail -20 $O/off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'])"; done
done
timeout -k 10 600 python3 -u -m pytest tests/test_tuning_gpu.py tests/test_transformer_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
echo done
