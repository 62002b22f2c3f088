#!/bin/bash
# joint (tile width, K-splits) plan of the linear weight gradients: sweep + tests + GPT-2 / ResNet-50 A/B vs ab_old
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_34
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
[ -s $O/sweep.txt ] || timeout -k 10 200 python3 dev/probes/wgrad_sweep.py 2>&1 | grep -v amdgpu.ids | tee $O/sweep.txt || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -v --timeout 170 --timeout-method thread -k "wgrad or pp or linear or gpt2" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in gpt2; do
    timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_new_$i.json 2> $O/${m}_new_$i.err || { tail -20 $O/${m}_new_$i.err; exit 1; }
    (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_old_$i.json 2> $O/${m}_old_$i.err) || { tail -20 $O/${m}_old_$i.err; exit 1; }
    for v in new old; do python3 -c "import json;d=json.load(open('$O/${m}_${v}_$i.json'));print('$m $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
  done
done
timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --diag-steps 0 > $O/resnet50_new.json 2> $O/resnet50_new.err || { tail -20 $O/resnet50_new.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/resnet50_new.json'));print('resnet50 new',d['value'],d['ms_per_step'],d['final_loss'])"
echo done
