#!/bin/bash
# transformer / graph / trajectory / kernel suites with the fused cross-entropy default
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_50
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_graphs_gpu.py tests/test_trajectory_gpu.py tests/test_ddp_gpu.py tests/test_tuning_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
