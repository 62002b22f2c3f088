#!/bin/bash
# epilogue pairing (pp_epi_pair) + packed bf16 conversions: bit-equality tests, per-GEMM A/B, K-sweep traces, GPT-2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_12
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_tuning_gpu.py -k "slack or narrow_tile or kernel_entry or pp_" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 dev/probes/epi_slack.py > $O/gemms.jsonl 2> $O/gemms.err || { tail -20 $O/gemms.err; exit 1; }
cat $O/gemms.jsonl
for pr in 0 1; do
  PDNN_TUNE=pp_epi_slack=1,pp_epi_pair=$pr timeout -k 10 60 python3 dev/probes/pp_one.py 8192 50304 768 --bn 288 --trace 2>&1 | grep -v amdgpu.ids | tee -a $O/trace.txt || exit 1
  PDNN_TUNE=pp_epi_slack=1,pp_epi_pair=$pr timeout -k 10 60 python3 dev/probes/pp_one.py 8192 50304 768 --bn 256 --trace 2>&1 | grep -v amdgpu.ids | tee -a $O/trace.txt || exit 1
done
run() {
  local n=$1; shift
  local m=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model $m --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run g00 gpt2_small PDNN_TUNE=pp_epi_slack=0,pp_epi_pair=0 && run g11 gpt2_small PDNN_TUNE=pp_epi_slack=1,pp_epi_pair=1 && run g00b gpt2_small PDNN_TUNE=pp_epi_slack=0,pp_epi_pair=0 && run g11b gpt2_small PDNN_TUNE=pp_epi_slack=1,pp_epi_pair=1 || exit 1
run r00 resnet50 PDNN_TUNE=pp_epi_slack=0,pp_epi_pair=0 && run r11 resnet50 PDNN_TUNE=pp_epi_slack=1,pp_epi_pair=1 || exit 1
echo done
