#!/bin/bash
# full GPU suite + smoke + ResNet-50 / GPT-2 benches after the PS / k-of-n / GEMM changes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_r50.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 20 --warmup 5 > $O/bench_gpt2.log 2>&1 || exit $?
