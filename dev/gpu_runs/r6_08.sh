#!/bin/bash
# ResNet-152 bf16 / fp8 kernel traces: which stream bounds the step (why fp8 3x3 convs pay only ~1%)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_08
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in bf16 fp8; do
  F=""; [ $v = fp8 ] && F="--fp8"
  timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/t_$v -o t_$v --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet152 --steps 4 --warmup 3 --plain $F > $O/$v.log 2>&1 || exit $?
  find /tmp/t_$v -name "*kernel_trace.csv" -exec cp {} $O/${v}_trace.csv \;
  python3 $GRAFT_REPO_ROOT/tools/stream_busy.py $O/${v}_trace.csv --top 14 > $O/${v}_busy.txt 2>&1
  head -40 $O/${v}_busy.txt
done
echo done
