#!/bin/bash
# host-side profile of one DDP-path step (1-rank RCCL): where the host stalls at the start of the backward
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_62
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29751 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1
timeout -k 10 200 python -u tools/ddp_host_profile.py --min-us 30 > $O/host.log 2>&1 || { tail -30 $O/host.log; exit 1; }
echo done
