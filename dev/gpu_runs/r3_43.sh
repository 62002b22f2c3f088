#!/bin/bash
# direct 3x3 weight gradient: numerics, per-layer wgrad table (vs MIOpen), step A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_43
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k wgrad > $O/pytest_w3.log 2>&1 || { tail -40 $O/pytest_w3.log; exit 1; }
tail -1 $O/pytest_w3.log
timeout -k 10 400 python -u tools/bench_conv.py --only wgrad --json $O/wg_default.json > $O/wg_default.log 2>&1 || { tail -20 $O/wg_default.log; exit 1; }
grep -v amdgpu.ids $O/wg_default.log | tail -30
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_blocks_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_trajectory_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for T in "" "wgrad3x3=0" "" "wgrad3x3=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
