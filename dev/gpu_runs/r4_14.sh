#!/bin/bash
# pp epilogue: bias hoisted per item, residual / dGELU operand prefetched one row ahead
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_14
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_transformer_gpu.py tests/test_kernels_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u dev/probes/epi_cost.py > $O/epi.log 2>&1 || { tail -20 $O/epi.log; exit 1; }
grep shape $O/epi.log
timeout -k 10 300 python -u bench.py --model gpt2_small --no-ddp-rehearsal > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 1; }
grep -o '"value": [0-9.]*, [^,]*, [^,]*, [^,]*, [^,]*, "ms_per_step": [0-9.]*' $O/gpt2.log
timeout -k 10 300 python -u bench.py --no-ddp-rehearsal > $O/r50.log 2>&1 || { tail -20 $O/r50.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r50.log
