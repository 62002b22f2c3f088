#!/bin/bash
# pp_dgrad_bn_k table entry: tuning battery, then same-box A/B of the ResNet-50 step (1024 vs off)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_17
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_tuning_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc
bash dev/probes/ab_bench.sh $O "pp_dgrad_bn_k=1024" "pp_dgrad_bn_k=1048576" 3
