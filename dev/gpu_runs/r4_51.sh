#!/bin/bash
# BN1 + ReLU applied while staging (no a1 materialisation): numerics (kernels, trajectories), ResNet-50 A/B vs HEAD,
# ResNet-152 bf16 / fp8 pair
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_51
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_fp8_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_trajectory_gpu.py tests/test_models_gpu.py > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
tail -2 $O/traj.log
bash dev/probes/ab_lib.sh $O/r50 pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 3 --steps 20 --warmup 8 || exit 1
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-110 $O/*.json
