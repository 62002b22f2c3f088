#!/bin/bash
# weight-stationary 1x1 kernel (K in {512, 1024}): numerics, per-layer, whole step A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_30
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py \
  tests/test_tuning_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for T in "breg=0" ""; do
  PDNN_TUNE="$T" timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/l1x1_$T.log 2>&1 || exit 1
  echo "[$T]"; cat $O/l1x1_$T.log | grep -v amdgpu.ids
done
i=0
for T in "" "breg=0" "" "breg=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
