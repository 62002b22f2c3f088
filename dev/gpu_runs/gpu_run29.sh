#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run29
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10 120"
$T python -u tools/graph_diag.py --batch 32 --style forward > $O/a.log 2>&1 || exit $?
$T python -u tools/graph_diag.py --batch 64 --style forward > $O/b.log 2>&1 || exit $?
$T python -u tools/graph_diag.py --batch 32 --style loss_fn > $O/c.log 2>&1 || exit $?
AMD_LOG_LEVEL=3 $T python -u tools/graph_diag.py --batch 64 --style loss_fn > $O/d.log 2>&1 || exit $?
