#!/bin/bash
# host-side profile of the DDP-path step; same-box A/B old commit vs bins (raw-stream pool key)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_06
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 dev/probes/host_profile.py > $O/host_profile.txt 2> $O/host_profile.err || { tail -20 $O/host_profile.err; exit 1; }
head -60 $O/host_profile.txt | tail -50
timeout -k 10 300 python3 tools/host_timing.py > $O/host_timing.txt 2>&1 || { tail -20 $O/host_timing.txt; exit 1; }
tail -12 $O/host_timing.txt
for i in 1 2; do
  (cd $R/ab_old && timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/old_$i.json 2> $O/old_$i.err) || { tail -20 $O/old_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --no-plain-run --diag-steps 0 > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  python3 -c "
import json
for v in ('old','new'):
    l=[x for x in open('$O/'+v+'_$i.json') if x.startswith('{')][-1]; print(v, json.loads(l)['value'])"
done
echo done
