#!/bin/bash
# attention backward with two 16-row fragments per wave (attn_bwd_wide bit mask): tests, kernel times, GPT-2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_45
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in 0 1 2 3; do
PDNN_TUNE=attn_bwd_wide=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "attention or flash" > $O/tests_$v.log 2>&1 || { tail -40 $O/tests_$v.log; exit 1; }
echo "wide=$v $(tail -1 $O/tests_$v.log)"
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tuning_gpu.py > $O/tuning.log 2>&1 || { tail -40 $O/tuning.log; exit 1; }
tail -1 $O/tuning.log
for v in 0 1 2 3; do
PDNN_TUNE=attn_bwd_wide=$v timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_$v.jsonl 2>&1 || { cat $O/attn_$v.jsonl; exit 1; }
echo "wide=$v"; grep causal $O/attn_$v.jsonl | cut -c1-120
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
for v in 0 1 3; do
run w${v}_$i PDNN_TUNE=attn_bwd_wide=$v || exit 1
done
done
echo done
