#!/bin/bash
# DDP bucket collectives (and the BN-buffer broadcast) issued from a DDP-owned launch stream: tests + A/B vs HEAD
# (ab_old worktree) + a GPT-2 kernel trace to check the backward block-boundary gaps
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_30
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for m in gpt2 resnet50; do
    timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_new_$i.json 2> $O/${m}_new_$i.err || { tail -20 $O/${m}_new_$i.err; exit 1; }
    (cd $R/ab_old && timeout -k 10 300 python3 bench.py --model $m --no-plain-run --diag-steps 0 > $O/${m}_old_$i.json 2> $O/${m}_old_$i.err) || { tail -20 $O/${m}_old_$i.err; exit 1; }
    for v in new old; do python3 -c "import json;d=json.load(open('$O/${m}_${v}_$i.json'));print('$m $v',d['value'],d['ms_per_step'],d['final_loss'])"; done
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g8 -o g8 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g8.log 2>&1 || exit $?
find /tmp/g8 -name "*kernel_trace.csv" -exec cp {} $O/g8_trace.csv \;
cd $R && python3 tools/prof_summary.py $O/g8_trace.csv --steps 3 --by-grid --top 50 > $O/grid_summary.txt 2>&1
head -12 $O/grid_summary.txt
echo done
