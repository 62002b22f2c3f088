#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/run6
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/run6/pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/run6/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 5 > gpurun_out/run6/bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_conv.py --no-ref --json gpurun_out/run6/bench_conv.json > gpurun_out/run6/bench_conv.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/run6/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/run6/prof.log 2>&1
