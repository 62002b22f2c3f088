#!/bin/bash
# ResNet-50 DDP-path kernel trace: per-stream split (current defaults)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_47
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g47 -o g47 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/g47.log 2>&1 || exit $?
find /tmp/g47 -name "*kernel_trace.csv" -exec cp {} $O/trace.csv \;
cd $R && python3 tools/stream_busy.py $O/trace.csv --step-kernel sgd_kernel --full --top 40 > $O/streams.txt 2>&1
cat $O/streams.txt | cut -c1-150
echo done
