#!/bin/bash
# xent backward scale from the device-side count: tests, ResNet-50 / GPT-2 bench; then host-lead trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_67
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[r50] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
timeout -k 10 300 python -u bench.py --model gpt2_small --steps 20 --no-ddp-rehearsal > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 1; }
echo "[gpt2] $(grep -o '"value": [0-9.]*' $O/gpt2.log)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/prof -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --no-ddp-rehearsal > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
ls $O/prof
echo done
