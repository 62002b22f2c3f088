#!/bin/bash
# stride-2 halo kernels + subsampled shortcuts: numerics tests, per-shape A/B vs the implicit-GEMM engine, fused
# block tests, ResNet-50 bench A/B of s2_halo / ds_sub
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_02
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_s2_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python3 tools/bench_conv_s2.py > $O/bench_s2.jsonl 2> $O/bench_s2.err || { tail -20 $O/bench_s2.err; exit 1; }
cat $O/bench_s2.jsonl
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_blocks_gpu.py > $O/fused.log 2>&1 || { tail -40 $O/fused.log; exit 1; }
tail -2 $O/fused.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-plain-run --no-extra-configs --diag-steps 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run s2_11 PDNN_TUNE=s2_halo=11 && run s2_0 PDNN_TUNE=s2_halo=0,ds_sub=0 && run ds0 PDNN_TUNE=ds_sub=0 && run s2_3 PDNN_TUNE=s2_halo=3 && run s2_15 PDNN_TUNE=s2_halo=15 && run s2_11b PDNN_TUNE=s2_halo=11 || exit 1
echo done
