#!/bin/bash
# attention backward: lse/delta through LDS, prologue loads drained before the loop, transposed fragments batched
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_34
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_transformer_gpu.py tests/test_kernels_gpu.py -k "attn or attention or flash or gpt" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn.py > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 1; }
PDNN_KERNEL_LIB=pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so timeout -k 10 200 python -u tools/bench_attn.py > $O/attn_base.log 2>&1 || { tail -20 $O/attn_base.log; exit 1; }
grep -h '{' $O/attn.log $O/attn_base.log | cut -c1-300
bash dev/probes/ab_lib.sh $O pytorch_distributed_nn_amd/_lib/ab/libpdnn_kernels_base.so 2 --model gpt2_small
