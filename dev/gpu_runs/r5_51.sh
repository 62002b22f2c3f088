#!/bin/bash
# positional-embedding gradient as an atomic-free per-position sum: tests + GPT-2 A/B vs ab_old (HEAD before it)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_51
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/old_$i.json 2> $O/old_$i.err) || { tail -20 $O/old_$i.err; exit 1; }
  for v in new old; do python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v',d['value'],d['ms_per_step'],d['final_loss'])"; done
done
echo done
