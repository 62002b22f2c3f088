#!/bin/bash
# attention forward: permlane row maxima, per-lane row sums, lazy rescale -- tests + kernel A/B vs HEAD lib + GPT-2
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_44
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "attention or flash" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_new.jsonl 2>&1 || { cat $O/attn_new.jsonl; exit 1; }
PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab_old/libpdnn_kernels.so timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_old.jsonl 2>&1 || { cat $O/attn_old.jsonl; exit 1; }
timeout -k 10 120 python3 tools/bench_attn.py > $O/attn_new2.jsonl 2>&1 || exit 1
grep causal $O/attn_old.jsonl $O/attn_new.jsonl $O/attn_new2.jsonl | cut -c1-200
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])"
}
for i in 1 2; do
run old_$i PDNN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab_old/libpdnn_kernels.so || exit 1
run new_$i || exit 1
done
echo done
