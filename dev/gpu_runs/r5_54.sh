#!/bin/bash
# native RCCL path on the two-stream ResNet-50: comm stream priority (diagnostic)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_54
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run nat_prio_hi PDNN_DDP_NATIVE_COMM=1 PDNN_NATIVE_COMM_PRIO=-1 && run pg PDNN_TUNE=side_wgrad=1 || exit 1
echo done
