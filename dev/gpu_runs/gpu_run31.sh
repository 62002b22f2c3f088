#!/bin/bash
# hipBLASLt probe for GPT-2 GEMM shapes + current GPT-2 kernel breakdown.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run31
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/blas_probe.py > $O/blas_probe.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_g2 -o g2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 4 --warmup 3 > $O/prof_g2.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py /tmp/prof_g2/g2_kernel_trace.csv --window-ms 80 --steps 3 --top 40 > $O/g2_summary.txt
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py /tmp/prof_g2/g2_kernel_trace.csv --window-ms 80 --steps 3 --top 60 --by-grid > $O/g2_summary_grid.txt
