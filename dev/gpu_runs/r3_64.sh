#!/bin/bash
# which stream is current in an autograd final callback under a non-default stream
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_64
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/callback_stream_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -1 $O/probe.log
