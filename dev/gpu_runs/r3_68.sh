#!/bin/bash
# stem weight gradient accumulated straight into the arena: stem / model / fused-block tests, bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_68
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py tests/test_models_gpu.py tests/test_fused_blocks_gpu.py tests/test_trajectory_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[r50] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
