#!/bin/bash
# Round-end rehearsal after a fresh in-tree rebuild: smoke(), full GPU suite, ResNet-50 + GPT-2 benches,
# rocprofv3 kernel stats of the flagship step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run59
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash): keep going
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model gpt2_small --steps 10 --warmup 3 > $O/bench_gpt2.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $O/prof.log 2>&1
