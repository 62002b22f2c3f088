#!/bin/bash
# K<=128 hand-off (no scratch), BN epilogue sums deferred to the flush (K=256 BNB variant out of scratch); A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_35
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_link_gpu.py tests/test_trajectory_gpu.py tests/test_fused_blocks_gpu.py tests/test_conv3x3_gpu.py tests/test_kernels_gpu.py tests/test_tuning_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for T in "" "bn_link=0" "wgrad1x1_pp_pix=0" "" "bn_link=0" "wgrad1x1_pp_pix=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
