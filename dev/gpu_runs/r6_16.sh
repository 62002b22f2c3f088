#!/bin/bash
# ResNet-50 routing log (which entry point each conv takes) + 1x1 forwards with C >= 512 on the ping-pong engine (A/B)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_16
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tuning_gpu.py -k "kernel_entry or table" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 dev/probes/route_log.py resnet50 256 > $O/route.txt 2> $O/route.err || { tail -20 $O/route.err; exit 1; }
cat $O/route.txt
run() {
  local n=$1; shift
  local m=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model $m --no-plain-run --no-extra-configs > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run r0 resnet50 PDNN_TUNE=pp_conv_fwd_c=1048576 && run r1 resnet50 PDNN_TUNE=pp_conv_fwd_c=512 && run r0b resnet50 PDNN_TUNE=pp_conv_fwd_c=1048576 && run r1b resnet50 PDNN_TUNE=pp_conv_fwd_c=512 || exit 1
echo done
