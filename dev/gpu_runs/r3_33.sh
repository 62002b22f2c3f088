#!/bin/bash
# batched-load BN slab finalize: BN tests + bench x2 + kernel trace; 1x1 wgrad engines (128-row vs ping-pong)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_33
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "bn or batchnorm or fused or block" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[b$i] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
timeout -k 10 300 python -u tools/bench_wgrad1x1.py > $O/wgrad1x1.log 2>&1 || { tail -20 $O/wgrad1x1.log; exit 1; }
grep -v amdgpu.ids $O/wgrad1x1.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof.log 2>&1 || exit 1
echo done
