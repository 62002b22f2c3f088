#!/bin/bash
# confirm the new glds defaults (dgrad on the 128-tile kernel, forward K >= 1024): smoke, GPU suite,
# ResNet-50 / ResNet-152 benches, rocprofv3 kernel stats
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run64
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
for rep in 1 2; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_$rep.log 2>&1 || exit $?; done
timeout -k 10 300 python -u bench.py --model resnet152 --steps 10 --warmup 3 > $O/bench_r152.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --graph off > $O/prof.log 2>&1
