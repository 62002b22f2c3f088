#!/bin/bash
# A/B: gemm_kernel register prefetch distance 2 (dev_lib/libpdnn_kernels_pf2.so) vs default; GPU suite on the variant
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_31
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/dev_lib/libpdnn_kernels_pf2.so
PDNN_KERNEL_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_pf2.log 2>&1
rc=$?; tail -n 3 $O/pytest_pf2.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 > $O/bench_base$i.log 2>&1 && tail -n 1 $O/bench_base$i.log | cut -c1-140 || exit 1
PDNN_KERNEL_LIB=$V timeout -k 10 200 python -u bench.py --steps 30 --warmup 8 > $O/bench_pf2_$i.log 2>&1 && tail -n 1 $O/bench_pf2_$i.log | cut -c1-140 || exit 1
done
PDNN_KERNEL_LIB=$V timeout -k 10 200 python -u bench.py --model resnet152 --steps 10 --warmup 5 > $O/bench_r152_pf2.log 2>&1 && tail -n 1 $O/bench_r152_pf2.log | cut -c1-140 || exit 1
cd /tmp && PDNN_KERNEL_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pf2 -o r50 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --graph off > $O/prof_pf2.log 2>&1 || exit 1
echo done
