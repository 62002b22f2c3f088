#!/bin/bash
# stride-2 halo kernels: numerics tests + per-shape A/B vs the implicit-GEMM engine + ResNet-50 bench with / without
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_02
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_s2_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python3 tools/bench_conv_s2.py > $O/bench_s2.jsonl 2> $O/bench_s2.err || { tail -20 $O/bench_s2.err; exit 1; }
cat $O/bench_s2.jsonl
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run s2_3 PDNN_TUNE=s2_halo=3 && run s2_0 PDNN_TUNE=s2_halo=0 && run s2_1 PDNN_TUNE=s2_halo=1 && run s2_7 PDNN_TUNE=s2_halo=7 && run s2_3b PDNN_TUNE=s2_halo=3 || exit 1
echo done
