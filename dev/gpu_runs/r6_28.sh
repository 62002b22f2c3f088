#!/bin/bash
# N = 1 DDP bucket caps (the all-reduce is a no-op there; each collective costs a stream-sync event): A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_28
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-plain-run --no-extra-configs --diag-steps 2 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d['comm']['bucket_mb'])"
}
for i in 1 2; do
run r32_$i --model resnet50 --bucket-mb 32 && run r64_$i --model resnet50 --bucket-mb 64 && run r128_$i --model resnet50 --bucket-mb 128 || exit 1
run g128_$i --model gpt2_small --bucket-mb 128 && run g256_$i --model gpt2_small --bucket-mb 256 && run g1024_$i --model gpt2_small --bucket-mb 1024 || exit 1
done
echo done
