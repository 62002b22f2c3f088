#!/bin/bash
# fp32-epilogue store slack (pp_epi_slack 2) on the GPT-2 weight gradients: bits, per-GEMM, end to end
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_13
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pp_wgrad or slack" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sl in 1 2 1 2; do
  for shp in "2304 768 8192" "768 768 8192" "3072 768 8192" "768 3072 8192" "50304 768 8192"; do
    PDNN_TUNE=pp_epi_slack=$sl timeout -k 10 60 python3 dev/probes/pp_one.py $shp --kind wgrad 2>&1 | grep -v amdgpu.ids | sed "s/^/slack$sl /" | tee -a $O/wgrad.txt || exit 1
  done
done
run() {
  local n=$1; shift
  local m=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model $m --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run g1 gpt2_small PDNN_TUNE=pp_epi_slack=1 && run g2 gpt2_small PDNN_TUNE=pp_epi_slack=2 && run g1b gpt2_small PDNN_TUNE=pp_epi_slack=1 && run g2b gpt2_small PDNN_TUNE=pp_epi_slack=2 || exit 1
run r1 resnet50 PDNN_TUNE=pp_epi_slack=1 && run r2 resnet50 PDNN_TUNE=pp_epi_slack=2 || exit 1
echo done
