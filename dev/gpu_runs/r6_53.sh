#!/bin/bash
# ResNet-50 DDP path: kernel trace + HIP runtime API trace -- are the compute stream's idle gaps host-bound?
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_53
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/g53 -o g53 --output-format csv -- python3 $R/bench.py --steps 4 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/g53.log 2>&1 || exit $?
find /tmp/g53 -name "*kernel_trace.csv" -exec cp {} $O/trace.csv \;
find /tmp/g53 -name "*hip_api_trace.csv" -exec cp {} $O/api.csv \;
ls -la $O
echo done
