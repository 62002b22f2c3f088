#!/bin/bash
# host enqueue time of one step (idle GPU at its start) vs its wall time, GPT-2 DDP path / plain and ResNet-50 DDP;
# cProfile of one GPT-2 DDP step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_56
mkdir -p $O
cd $GRAFT_REPO_ROOT
PDNN_BENCH_HOST_PROBE=2 timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs --no-plain-run > $O/g_ddp.json 2> $O/g_ddp.err || { tail -20 $O/g_ddp.err; exit 1; }
PDNN_BENCH_HOST_PROBE=1 timeout -k 10 300 python3 bench.py --model gpt2_small --no-extra-configs --plain > $O/g_plain.json 2> $O/g_plain.err || { tail -20 $O/g_plain.err; exit 1; }
PDNN_BENCH_HOST_PROBE=2 timeout -k 10 300 python3 bench.py --no-extra-configs --no-plain-run > $O/r_ddp.json 2> $O/r_ddp.err || { tail -20 $O/r_ddp.err; exit 1; }
for f in g_ddp g_plain r_ddp; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],d.get('host_probe'))"; done
echo done
