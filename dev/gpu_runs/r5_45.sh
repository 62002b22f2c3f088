#!/bin/bash
# ResNet-50 plain step: hipGraph replay (two-stream schedule captured) vs eager, ROCm 7.2 (r2_32 had the graph serialise the streams)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_45
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for g in on off; do
    timeout -k 10 300 python3 bench.py --plain --graph $g > $O/r50_${g}_$i.json 2> $O/r50_${g}_$i.err || { tail -20 $O/r50_${g}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/r50_${g}_$i.json'));print('graph $g',d['value'],d['ms_per_step'],d['config'].get('hipgraph'))"
  done
done
echo done
