#!/bin/bash
# split-K weight gradients with atomic partial adds instead of slabs + reduce: sweep + tests + A/B (PDNN_TUNE)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_39
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
PDNN_TUNE=pp_wgrad_atomic=1 timeout -k 10 200 python3 dev/probes/wgrad_sweep.py 2>&1 | grep -v amdgpu.ids | tee $O/sweep_atomic.txt || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_tuning_gpu.py tests/test_kernels_gpu.py -x -v --timeout 170 --timeout-method thread -k "wgrad or atomic" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in gpt2 resnet50; do
    PDNN_TUNE=pp_wgrad_atomic=1 timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_new_$i.json 2> $O/${m}_new_$i.err || { tail -20 $O/${m}_new_$i.err; exit 1; }
    timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_off_$i.json 2> $O/${m}_off_$i.err || { tail -20 $O/${m}_off_$i.err; exit 1; }
    for v in new off; do python3 -c "import json;d=json.load(open('$O/${m}_${v}_$i.json'));print('$m $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
  done
done
echo done
