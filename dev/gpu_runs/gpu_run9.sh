#!/bin/bash
# transformer kernels first (new code), then the full GPU suite, ResNet-50 bench, GPT-2 bench
set -o pipefail
O=gpurun_out/run9
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash): keep going
timeout -k 10 400 python -m pytest tests/test_transformer_gpu.py -q -x > $O/pytest_tx.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest_tx.log; ok $rc || exit $rc
timeout -k 10 700 python -m pytest tests/ -q -m gpu > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model gpt2_small --steps 10 --warmup 3 > $O/bench_gpt2.log 2>&1 || exit $?
