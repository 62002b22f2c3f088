#!/bin/bash
# PMC counters of the conv kernels (kernel-trace + pmc only; no sys/runtime trace)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run15
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
P="python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --no-ref --iters 2 --layers 3,16,7"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $O/pmc1 -o p1 --output-format csv -- $P > $O/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE -d $O/pmc2 -o p2 --output-format csv -- $P > $O/pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum -d $O/pmc3 -o p3 --output-format csv -- $P > $O/pmc3.log 2>&1 || exit $?
