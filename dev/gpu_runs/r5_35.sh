#!/bin/bash
# non-temporal stores for >= 256 MiB ping-pong bf16 outputs (GPT-2 LM-head logits): probe + tests + A/B (PDNN_TUNE)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_35
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
P=dev/probes/pp_one.py
timeout -k 10 60 python3 $P 8192 50304 768 --trace 2>&1 | grep -v amdgpu.ids | tee $O/fwd.txt || exit 1
PDNN_TUNE=pp_nt_mb=0 timeout -k 10 60 python3 $P 8192 50304 768 --trace 2>&1 | grep -v amdgpu.ids | tee -a $O/fwd.txt || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_tuning_gpu.py -x -v --timeout 170 --timeout-method thread -k "pp or nt_mb" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in gpt2 resnet50; do
    timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_new_$i.json 2> $O/${m}_new_$i.err || { tail -20 $O/${m}_new_$i.err; exit 1; }
    PDNN_TUNE=pp_nt_mb=0 timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_off_$i.json 2> $O/${m}_off_$i.err || { tail -20 $O/${m}_off_$i.err; exit 1; }
    for v in new off; do python3 -c "import json;d=json.load(open('$O/${m}_${v}_$i.json'));print('$m $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
  done
done
echo done
