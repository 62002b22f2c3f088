#!/bin/bash
# native RCCL bucket path on ResNet-50: is the slowdown tied to the weight-gradient side stream? (diagnostic)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_53
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run pg_side PDNN_TUNE=side_wgrad=1 && run nat_side PDNN_DDP_NATIVE_COMM=1 && run pg_noside PDNN_TUNE=side_wgrad=0 && run nat_noside PDNN_TUNE=side_wgrad=0 PDNN_DDP_NATIVE_COMM=1 || exit 1
echo done
