#!/bin/bash
# direct 3x3 wgrad, padded halo with immediate tap offsets: ablations, numerics, step A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_46
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/w3_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k wgrad > $O/pytest_w3.log 2>&1 || { tail -40 $O/pytest_w3.log; exit 1; }
tail -1 $O/pytest_w3.log
i=0
for T in "" "wgrad3x3=0" "" "wgrad3x3=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
