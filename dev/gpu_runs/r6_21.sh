#!/bin/bash
# A-stationary 1x1 kernel: cost of the statistics epilogue
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_21
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 dev/probes/areg_stats_cost.py > $O/areg.jsonl 2> $O/areg.err || { tail -20 $O/areg.err; exit 1; }
cat $O/areg.jsonl
echo done
