#!/bin/bash
# fused cross-entropy: gradient parity with the two-pass form at a GPT-2 vocabulary (device-alpha GEMM path)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_26
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 170 --timeout-method thread -k "fused_cross or xent" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 170 --timeout-method thread -k "xent" >> $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
timeout -k 10 300 python3 dev/probes/xent_traj.py --ddp > $O/traj_ddp.txt 2>&1; grep -v amdgpu.ids $O/traj_ddp.txt | head -5
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  PDNN_TUNE=xent_fused=0 timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/off_$i.json 2> $O/off_$i.err || { tail -20 $O/off_$i.err; exit 1; }
  for v in new off; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
