#!/bin/bash
# locate the address-dependent mismatch (r6_04): first kernel call whose output differs between two model copies
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_05
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 dev/probes/det_trace.py > $O/trace.log 2>&1 || { tail -30 $O/trace.log; exit 1; }
grep -v "^\[W\|amdgpu.ids" $O/trace.log
echo done
