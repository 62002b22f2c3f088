#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/run3
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_models_gpu.py -x -q -m gpu > gpurun_out/run3/pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/run3/pytest.log
timeout -k 10 400 python bench.py --steps 10 --warmup 5 > gpurun_out/run3/bench.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/run3/prof -o ours --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/run3/prof.log 2>&1
