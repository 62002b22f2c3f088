#!/bin/bash
# full GPU suite after the ping-pong epilogue / split-K / 1x1-forward routing changes, then smoke()
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_18
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo done
