#!/bin/bash
# fp8 ResNet-50 memorisation loss curves: current kernels vs the session-start build (4e4085c)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_25
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u dev/probes/fp8_train_probe.py > $O/cur.log 2>&1 || { tail -20 $O/cur.log; exit 1; }
grep fp8 $O/cur.log
PDNN_KERNEL_LIB=pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so timeout -k 10 300 python -u dev/probes/fp8_train_probe.py > $O/base.log 2>&1 || { tail -20 $O/base.log; exit 1; }
grep fp8 $O/base.log
