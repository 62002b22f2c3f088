#!/bin/bash
# full GPU suite + smoke on the current tree
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_42
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
