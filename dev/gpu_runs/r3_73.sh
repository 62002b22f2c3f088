#!/bin/bash
# wprep_once (one side fork per forward, one compute-stream wait per backward): tests + A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_73
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_blocks_gpu.py tests/test_models_gpu.py tests/test_trajectory_gpu.py tests/test_ddp_gpu.py tests/test_graphs_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for T in "" "wprep_once=0" "" "wprep_once=0" "" "wprep_once=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
