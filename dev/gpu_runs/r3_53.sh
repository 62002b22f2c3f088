#!/bin/bash
# padded partial / slab strides (HBM channel camping): tests, step, GPT-2, trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_53
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_kernels_gpu.py tests/test_transformer_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1; echo "[b$i] $(grep -o '"value": [0-9.]*' $O/b$i.log)"; done
timeout -k 10 300 python -u bench.py --model gpt2_small --steps 20 --no-ddp-rehearsal > $O/gpt2.log 2>&1 || exit 1
echo "[gpt2] $(grep -o "\"value\": [0-9.]*" $O/gpt2.log)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof.log 2>&1 || exit 1
echo done
