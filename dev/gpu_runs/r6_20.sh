#!/bin/bash
# 1x1 forwards with C <= 256 (no prologue) on the ping-pong engine instead of the A-stationary kernel (A/B), +tests
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_20
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tuning_gpu.py -k "python_entry" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for i in 1 2; do
run base$i PDNN_TUNE=areg_fwd=1 && run pp64_$i PDNN_TUNE=areg_fwd=0,pp_conv_fwd_c=64 && run pp256_$i PDNN_TUNE=areg_fwd=0,pp_conv_fwd_c=256 || exit 1
done
echo done
