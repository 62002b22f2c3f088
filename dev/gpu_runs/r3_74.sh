#!/bin/bash
# end-state validation: full GPU suite, smoke, ResNet-50 bench (plain + DDP rehearsal), GPT-2 bench;
# final rocprof timeline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_74
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log
timeout -k 10 300 python -u bench.py --model gpt2_small --steps 20 --no-ddp-rehearsal > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 1; }
grep -o '"value": [0-9.]*' $O/gpt2.log
echo done
