#!/bin/bash
# 64-deep slices on the fused ping-pong variants (1x1 conv stats / prologue / BN-backward epilogues): numerics +
# ResNet-50 A/B (pp_sk64 = 1 vs 0) + GPT-2
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_20
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_tuning_gpu.py tests/test_fused_blocks_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=pp_sk64=0 timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/off_$i.json 2> $O/off_$i.err || { tail -20 $O/off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'])"; done
done
timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/g.json 2> $O/g.err || { tail -20 $O/g.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/g.json'));print('gpt2',d['value'],d['ms_per_step'])"
echo done
