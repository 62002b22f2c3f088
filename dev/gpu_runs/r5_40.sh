#!/bin/bash
# LayerNorm fwd / bwd bandwidth vs block count; end-state GPT-2 kernel trace (profile)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_40
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python3 dev/probes/ln_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/ln.txt || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g10 -o g10 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g10.log 2>&1 || exit $?
find /tmp/g10 -name "*kernel_trace.csv" -exec cp {} $O/g10_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g10_trace.csv --steps 3 --by-grid --top 60 > $O/grid_summary.txt 2>&1
head -5 $O/grid_summary.txt
echo done
