#!/bin/bash
# GPT-2 DDP path: bucket size (each collective's stream-sync event record idles the compute stream ~21 us, r5_40/43)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_44
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for mb in 32 64 128 256; do
    timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 --bucket-mb $mb > $O/b${mb}_$i.json 2> $O/b${mb}_$i.err || { tail -20 $O/b${mb}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${mb}_$i.json'));print('bucket_mb $mb',d['value'],d['ms_per_step'],d['final_loss'])"
  done
done
echo done
