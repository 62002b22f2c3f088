#!/bin/bash
# class-pair s2 dgrad + a1 by-product: numerics, guard, per-shape timing, step A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_06
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_s2_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 dev/probes/s2_guard.py 1 > $O/guard.log 2>&1 || { tail -30 $O/guard.log; exit 1; }
tail -1 $O/guard.log
timeout -k 10 200 python3 tools/bench_conv_s2.py > $O/bench_s2.jsonl 2> $O/bench_s2.err || { tail -20 $O/bench_s2.err; exit 1; }
cat $O/bench_s2.jsonl
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-plain-run --no-extra-configs --diag-steps 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run s67_$i PDNN_TUNE=s2_halo=67 && run s195_$i PDNN_TUNE=s2_halo=195 && run s3_$i PDNN_TUNE=s2_halo=3 && run s0_$i PDNN_TUNE=s2_halo=0 && run s131_$i PDNN_TUNE=s2_halo=131 || exit 1
done
echo done
