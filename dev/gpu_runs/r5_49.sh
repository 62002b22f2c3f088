#!/bin/bash
# ResNet-50 DDP path with the native RCCL bucket path: kernel trace (where do the 9 ms/step go?)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_49
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
PDNN_DDP_NATIVE_COMM=1 timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g13 -o g13 --output-format csv -- python3 $R/bench.py --steps 4 --warmup 3 --no-plain-run --diag-steps 0 > $O/g13.log 2>&1 || exit $?
find /tmp/g13 -name "*kernel_trace.csv" -exec cp {} $O/g13_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g13_trace.csv --steps 3 --by-grid --top 20 > $O/grid_summary.txt 2>&1
head -12 $O/grid_summary.txt
echo done
