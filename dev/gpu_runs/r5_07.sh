#!/bin/bash
# attention: global heavy-first block order (new default) vs per-(head, seq) order (o0 variant); GPT-2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_07
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_new.jsonl 2>&1 || exit 1
PDNN_KERNEL_LIB=$R/dev_lib/libpdnn_kernels_o0.so timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_o0.jsonl 2>&1 || exit 1
cut -c1-140 $O/attn_new.jsonl $O/attn_o0.jsonl | grep fwd_us
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/g_new_$i.json 2> $O/g_new_$i.err || { tail -5 $O/g_new_$i.err; exit 1; }
  PDNN_KERNEL_LIB=$R/dev_lib/libpdnn_kernels_o0.so timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/g_o0_$i.json 2> $O/g_o0_$i.err || { tail -5 $O/g_o0_$i.err; exit 1; }
  python3 -c "
import json
for v in ('new','o0'):
    d=json.load(open('$O/g_'+v+'_$i.json')); print(v, d['value'], d['config']['hipgraph'])"
done
echo done
