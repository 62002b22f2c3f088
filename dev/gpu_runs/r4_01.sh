#!/bin/bash
# round-4 baseline: flagship bench (+ DDP rehearsal with the new comm block) on this round's box; new DDP / PS
# GPU tests; K>=512 1x1 data-gradient layers under the three engines
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_01
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-300
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_default.log 2>&1 || { tail -20 $O/c1_default.log; exit 1; }
PDNN_TUNE=pp_conv_bnb_k=512 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_ppbnb.log 2>&1 || { tail -20 $O/c1_ppbnb.log; exit 1; }
PDNN_TUNE=glds_dgrad_k=512,glds_dgrad_n=64 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_glds.log 2>&1 || { tail -20 $O/c1_glds.log; exit 1; }
tail -n 1 $O/c1_*.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ddp_gpu.py tests/test_straggler_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo done
