#!/bin/bash
# Post-restore check: GPU tests, smoke, 1-GPU bench (ResNet-50 + GPT-2).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run26
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
