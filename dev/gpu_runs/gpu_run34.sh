#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run34
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python tools/bench_attn.py > $O/attn.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_r50_a.log 2>&1 || exit $?
$T 300 python bench.py > $O/bench_r50_b.log 2>&1 || exit $?
