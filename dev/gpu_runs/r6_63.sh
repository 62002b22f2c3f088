#!/bin/bash
# final full GPU suite, smoke, driver-shaped bench (attn_bwd_wide default 3)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_63
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t0=$(date +%s)
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "wall $(( $(date +%s) - t0 )) s"
python3 -c "
import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],d['ms_per_step'],'plain',d['plain_step_1gpu']['value'])
for k,v in (d.get('extra_configs') or {}).items(): print(k, v.get('value'), v.get('ms_per_step'), v.get('wall_s'), v.get('error'))"
echo done
