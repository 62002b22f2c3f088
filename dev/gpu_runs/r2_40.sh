#!/bin/bash
# masked-residual dgrad epilogue (no materialised masked shortcut gradient): full suite, A/B bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_40
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -n 8; [ $rc -le 1 ] || exit $rc
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 30 > $O/b_$n.log 2>&1 && echo "$n $(tail -n 1 $O/b_$n.log | cut -c60-110)" || exit 1; }
for i in 1 2; do
run mres$i PDNN_X=0
run nomres$i PDNN_MASK_RES=0
done
echo done
