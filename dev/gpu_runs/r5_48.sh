#!/bin/bash
# native RCCL bucket all-reduces (rccl_native.py): tests + GPT-2 (32 MB buckets: 13 collectives) and ResNet-50 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_48
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for cfg in "gpt2 32" "gpt2 128" "resnet50 32"; do
    set -- $cfg
    PDNN_DDP_NATIVE_COMM=1 timeout -k 10 300 python3 bench.py --model $1 --bucket-mb $2 --no-plain-run --diag-steps 0 > $O/${1}_${2}_nat_$i.json 2> $O/${1}_${2}_nat_$i.err || { tail -20 $O/${1}_${2}_nat_$i.err; exit 1; }
    timeout -k 10 300 python3 bench.py --model $1 --bucket-mb $2 --no-plain-run --diag-steps 0 > $O/${1}_${2}_pg_$i.json 2> $O/${1}_${2}_pg_$i.err || { tail -20 $O/${1}_${2}_pg_$i.err; exit 1; }
    for v in nat pg; do python3 -c "import json;d=json.load(open('$O/${1}_${2}_${v}_$i.json'));print('$1 $2 $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
  done
done
echo done
