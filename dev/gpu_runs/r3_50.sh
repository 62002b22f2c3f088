#!/bin/bash
# re-check the panel/areg dgrad test (numerics failure in r3_49)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_50
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k "panel" > $O/pytest.log 2>&1; tail -15 $O/pytest.log
