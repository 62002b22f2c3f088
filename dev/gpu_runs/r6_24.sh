#!/bin/bash
# stem backward tail in isolation (warm / cold caches)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_24
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 dev/probes/stem_bwd_cost.py > $O/stem.json 2> $O/stem.err || { tail -20 $O/stem.err; exit 1; }
cat $O/stem.json
echo done
