#!/bin/bash
# Round-5 end state: full GPU suite, smoke, bench (ResNet-50 DDP path + plain, GPT-2), ResNet-152 bf16 / fp8 pair
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_final3
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python3 bench.py > $O/bench_r50.json 2> $O/bench_r50.err || { tail -20 $O/bench_r50.err; exit 1; }
cut -c1-400 $O/bench_r50.json
timeout -k 10 400 python3 bench.py --model gpt2 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || { tail -20 $O/bench_gpt2.err; exit 1; }
cut -c1-300 $O/bench_gpt2.json
timeout -k 10 400 python3 bench.py --model resnet152 --no-plain-run --diag-steps 0 > $O/bench_r152.json 2> $O/bench_r152.err || { tail -20 $O/bench_r152.err; exit 1; }
timeout -k 10 400 python3 bench.py --model resnet152 --fp8 --no-plain-run --diag-steps 0 > $O/bench_r152_fp8.json 2> $O/bench_r152_fp8.err || { tail -20 $O/bench_r152_fp8.err; exit 1; }
for f in bench_r152 bench_r152_fp8; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
echo done
