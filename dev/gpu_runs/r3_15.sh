#!/bin/bash
# A-stationary 1x1 kernel (tuning areg) + mask16 halo staging: numerics, per-layer and whole-step A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_15
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for T in "areg=0" "" "areg=2"; do
  PDNN_TUNE="$T" timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/l1x1_$T.log 2>&1 || exit 1
  echo "[$T] $(tail -1 $O/l1x1_$T.log)"
done
i=0
for T in "" "areg=0" "areg=2" "" "areg=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
