#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run30
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_graphs_gpu.py -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for s in 1 2; do
  for g in off on; do
    $T 300 python bench.py --model resnet50_cifar --graph $g --steps 20 --warmup 5 > $O/bench_r50c_${g}_$s.log 2>&1 || exit $?
  done
done
