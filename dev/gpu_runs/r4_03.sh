#!/bin/bash
# long-reduction 1x1 kernel v2 (per-wave register ring): numerics, per-layer timings, whole-step A/B; folded
# dispatch table (tuning GPU tests); DDP / PS GPU tests
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_03
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv1x1_wide_gpu.py tests/test_conv3x3_gpu.py tests/test_stem_gpu.py > $O/pytest_wide.log 2>&1 || { tail -40 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_new.log 2>&1 || { tail -20 $O/c1_new.log; exit 1; }
grep '"H"' $O/c1_new.log | cut -c1-400
for v in "wide1x1_fwd=0,wide1x1_dgrad=0,bn3_pre=0" "bn3_pre=0" "wide1x1_fwd=0" "wide1x1_dgrad=0,bn3_pre=0" "" ; do
  PDNN_TUNE=$v timeout -k 10 200 python -u bench.py --no-ddp-rehearsal > "$O/bench_$v.log" 2>&1 || { tail -20 "$O/bench_$v.log"; exit 1; }
  echo "[$v] $(grep -o '"value": [0-9.]*' "$O/bench_$v.log")"
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_straggler_gpu.py tests/test_ddp_gpu.py tests/test_tuning_gpu.py tests/test_fused_blocks_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo done
