#!/bin/bash
# re-entry check on a fresh box: full GPU suite, smoke, default bench, GPT-2 / ResNet-152 (bf16, fp8) benches,
# ResNet-50 kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_30
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 20
[ $rc -le 1 ] || { echo "pytest exit $rc: stopping"; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -n 20 $O/smoke.log; exit 1; }
timeout -k 10 200 python -u bench.py > $O/bench_default.log 2>&1 && tail -n 1 $O/bench_default.log || exit 1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 > $O/bench_r50.log 2>&1 && tail -n 1 $O/bench_r50.log || exit 1
timeout -k 10 200 python -u bench.py --model gpt2_small --steps 30 --warmup 5 > $O/bench_gpt2.log 2>&1 && tail -n 1 $O/bench_gpt2.log || exit 1
timeout -k 10 200 python -u bench.py --model gpt2_small --fp8 --steps 30 --warmup 5 > $O/bench_gpt2_fp8.log 2>&1 && tail -n 1 $O/bench_gpt2_fp8.log || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --steps 10 --warmup 5 > $O/bench_r152.log 2>&1 && tail -n 1 $O/bench_r152.log || exit 1
timeout -k 10 200 python -u bench.py --model resnet152 --fp8 --steps 10 --warmup 5 > $O/bench_r152_fp8.log 2>&1 && tail -n 1 $O/bench_r152_fp8.log || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r50 -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --graph off > $O/prof_r50.log 2>&1 || exit 1
echo done
