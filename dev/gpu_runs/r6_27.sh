#!/bin/bash
# driver-shaped bench record after the round-6 ping-pong / statistics / stem changes, plus a ResNet-152 bf16 / fp8 pair
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_27
mkdir -p $O
cd $GRAFT_REPO_ROOT
t0=$(date +%s)
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "wall $(( $(date +%s) - t0 )) s"
cat $O/bench.json
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model resnet152 --no-plain-run --no-extra-configs > $O/r152_bf16_$i.json 2> $O/r152_bf16_$i.err || { tail -20 $O/r152_bf16_$i.err; exit 1; }
timeout -k 10 300 python3 bench.py --model resnet152 --fp8 --no-plain-run --no-extra-configs > $O/r152_fp8_$i.json 2> $O/r152_fp8_$i.err || { tail -20 $O/r152_fp8_$i.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r152_bf16_$i.json'));b=json.load(open('$O/r152_fp8_$i.json'));print('r152 bf16',a['value'],'fp8',b['value'],'ratio',round(b['value']/a['value'],4))"
done
echo done
