#!/bin/bash
# host-side launch cost: primitive costs, host vs GPU per step, per-phase host timeline; flagship per-tensor
# first-step gradients vs fp32 torch; bench with the raw-stream / cached-symbol launch path
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_06
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_trajectory_gpu.py -k flagship > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u dev/probes/host_prims.py > $O/prims.log 2>&1 || { tail -20 $O/prims.log; exit 1; }
tail -1 $O/prims.log
timeout -k 10 200 python -u tools/host_overhead.py > $O/host_overhead.log 2>&1 || { tail -20 $O/host_overhead.log; exit 1; }
tail -1 $O/host_overhead.log
timeout -k 10 200 python -u tools/host_timing.py > $O/host_timing.log 2>&1 || { tail -20 $O/host_timing.log; exit 1; }
tail -8 $O/host_timing.log
timeout -k 10 400 python -u bench.py --no-ddp-rehearsal > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench.log
echo done
