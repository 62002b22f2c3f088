#!/bin/bash
# final end-of-round validation: full GPU suite, smoke, driver-style bench (defaults), GPT-2 bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_58
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python3 bench.py --model gpt2_small --steps 20 --warmup 8 > $O/gpt2.json 2> $O/gpt2.err || { tail -20 $O/gpt2.err; exit 1; }
cut -c1-200 $O/gpt2.json
