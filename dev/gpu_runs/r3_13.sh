#!/bin/bash
# BN-backward apply fused into the halo / panel data-gradient loads: numerics, model A/B, bench A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_13
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py \
  "tests/test_tuning_gpu.py::test_python_entry_alternatives" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for T in "" "bwd_pre=0" "" "bwd_pre=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
