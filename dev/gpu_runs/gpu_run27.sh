#!/bin/bash
# hipGraph step: graph tests, Adam kernel test, eager vs graph benches (headline + reference small configs).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run27
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_graphs_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "graph or sgd or adam" > $O/pytest.log 2>&1 || exit $?
for m in resnet50 gpt2_small lenet resnet18_cifar resnet50_cifar; do
  for g in off on; do
    $T 300 python bench.py --model $m --graph $g --steps 20 --warmup 5 > $O/bench_${m}_${g}.log 2>&1 || exit $?
  done
done
$T 300 python tools/host_overhead.py --model resnet50 > $O/host_resnet50.log 2>&1 || exit $?
$T 300 python tools/host_overhead.py --model gpt2_small > $O/host_gpt2.log 2>&1 || exit $?
