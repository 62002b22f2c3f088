#!/bin/bash
# LayerNorm backward grid sweep (GPT-2 shape)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_19
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 dev/probes/ln_bwd_grid.py > $O/ln.json 2> $O/ln.err || { tail -20 $O/ln.err; exit 1; }
cat $O/ln.json
echo done
