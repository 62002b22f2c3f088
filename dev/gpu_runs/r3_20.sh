#!/bin/bash
# areg PRE prologue: LDS coefficient table, batched operand loads
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_20
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/l1x1.log 2>&1 || exit 1
cat $O/l1x1.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "$(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
echo done
