#!/bin/bash
# side-stream wgrad test (lockstep form)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_34
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_fused_blocks_gpu.py -q -k side_stream --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 15 $O/pytest.log; exit $rc
