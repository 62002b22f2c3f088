#!/bin/bash
# k-of-n (no straggler) tax vs the plain DDP path at world 1, with its parts switched off one at a time
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_10
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 dev/probes/kofn_tax.py > $O/kofn.log 2>&1 || { tail -20 $O/kofn.log; exit 1; }
grep '^{' $O/kofn.log
