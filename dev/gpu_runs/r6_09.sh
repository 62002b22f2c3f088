#!/bin/bash
# deferred epilogue-store drain (pp_epi_slack): bit-equality tests, per-GEMM A/B on GPT-2 shapes, GPT-2 / ResNet-50 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_09
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "epilogue_store_slack or narrow_tile" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 dev/probes/epi_slack.py > $O/gemms.jsonl 2> $O/gemms.err || { tail -20 $O/gemms.err; exit 1; }
cat $O/gemms.jsonl
run() {
  local n=$1; shift
  local m=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model $m --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run g0 gpt2_small PDNN_TUNE=pp_epi_slack=0 && run g1 gpt2_small PDNN_TUNE=pp_epi_slack=1 && run g0b gpt2_small PDNN_TUNE=pp_epi_slack=0 && run g1b gpt2_small PDNN_TUNE=pp_epi_slack=1 || exit 1
run r0 resnet50 PDNN_TUNE=pp_epi_slack=0 && run r1 resnet50 PDNN_TUNE=pp_epi_slack=1 || exit 1
echo done
