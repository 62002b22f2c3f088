#!/bin/bash
# GPT-2 eager plain step (no DDP, no graph) vs DDP path: where the block-boundary idle gaps come from
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_43
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model gpt2 --plain --graph off > $O/plain_eager_$i.json 2> $O/plain_eager_$i.err || { tail -20 $O/plain_eager_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/ddp_$i.json 2> $O/ddp_$i.err || { tail -20 $O/ddp_$i.err; exit 1; }
  for v in plain_eager ddp; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'],d['config'].get('hipgraph'))"; done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g11 -o g11 --output-format csv -- python3 $R/bench.py --model gpt2 --plain --graph off --steps 5 --warmup 3 > $O/g11.log 2>&1 || exit $?
find /tmp/g11 -name "*kernel_trace.csv" -exec cp {} $O/g11_trace.csv \;
echo done
