#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run21
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_lowk.py > $O/exp_a.log 2>&1 || exit $?
PDNN_LOWK_BN64=1 timeout -k 10 300 python tools/exp_lowk.py > $O/exp_b.log 2>&1 || exit $?
PDNN_GLDS=0 PDNN_LOWK_BN64=1 timeout -k 10 400 python tools/bench_conv.py --no-ref --only fwd --json $O/conv_b.json > $O/conv_b.log 2>&1 || exit $?
PDNN_GLDS=0 timeout -k 10 400 python tools/bench_conv.py --no-ref --only fwd --json $O/conv_a.json > $O/conv_a.log 2>&1 || exit $?
PDNN_LOWK_BN64=1 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_b.log 2>&1 || exit $?
