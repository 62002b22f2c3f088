#!/bin/bash
# kernel trace of the step with the direct 3x3 weight gradient
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_48
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && for i in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1; echo "[b$i] $(grep -o '"value": [0-9.]*' $O/b$i.log)"; done
echo done
