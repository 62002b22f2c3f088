#!/bin/bash
# bench: DDP path as the N=1 headline + plain step; CLI north-star path (lazy phase events, device-resident synthetic data) vs bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_03
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 400 python3 bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));r=d['plain_step_1gpu'];print(d['value'],r.get('value'),r.get('error'),json.dumps((d.get('comm') or {}).get('fp32')))"
done
export PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
timeout -k 10 400 python3 -m pytorch_distributed_nn_amd.cli --mode ddp --network resnet50 --dataset ImageNet --synthetic \
  --batch-size 256 --max-steps 50 --log-interval 10 --lr 0.1 --momentum 0.9 --weight-decay 5e-5 --metrics $O/cli.jsonl \
  --out-dir $O/out > $O/cli.log 2>&1 || { tail -30 $O/cli.log; exit 1; }
tail -3 $O/cli.log
python3 tools/cli_vs_bench.py $O/cli.jsonl $O/bench_2.json | tee $O/cli_vs_bench.json
echo done
