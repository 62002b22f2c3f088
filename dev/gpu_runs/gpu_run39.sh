#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run39
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_r50.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small > $O/bench_gpt2.log 2>&1 || exit $?
