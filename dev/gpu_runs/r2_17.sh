#!/bin/bash
# pp engine: 1x1 conv fusions (prologue, BN stats, BN-backward) -- numerics, per-layer, whole step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_17
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv or gemm" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u tools/bench_conv.py --batch 256 --no-ref --json $O/conv_layers.json > $O/conv.log 2>&1 && tail -5 $O/conv.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && tail -1 $O/bench.log
