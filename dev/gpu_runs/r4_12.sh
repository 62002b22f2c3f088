#!/bin/bash
# GELU epilogues on v_exp/v_rcp: GEMM / transformer numerics, GPT-2 bench + breakdown
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_12
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_transformer_gpu.py tests/test_kernels_gpu.py -k "gelu or gpt or transformer or attn or linear" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --model gpt2_small --no-ddp-rehearsal > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 1; }
grep -o '"value": [0-9.]*, [^,]*, [^,]*, [^,]*, [^,]*, "ms_per_step": [0-9.]*' $O/gpt2.log
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g4 -o g4 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt2_small --steps 4 --warmup 2 --no-ddp-rehearsal --graph off > $O/g4.log 2>&1 || exit $?
find /tmp/g4 -name "*kernel_trace.csv" -exec cp {} $O/g4_trace.csv \;
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $O/g4_trace.csv --steps 3 --by-grid --top 50 > $O/g4_summary.txt 2>&1
head -12 $O/g4_summary.txt | cut -c1-200
