#!/bin/bash
# split-count sweeps with the paired epilogues: LM-head data gradient (uneven splits) and the GPT-2 weight gradients
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_15
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 dev/probes/splitk_sweep.py > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model gpt2_small --no-plain-run --no-extra-configs > $O/g$i.json 2> $O/g$i.err || { tail -20 $O/g$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/g$i.json'));print('g$i',d['value'],d['ms_per_step'])"
done
echo done
