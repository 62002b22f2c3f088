#!/bin/bash
# one-instruction fragment statistics atomics: numerics (kernel / fused-block / tuning suites), areg cost, ResNet A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_22
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_blocks_gpu.py tests/test_tuning_gpu.py tests/test_conv_s2_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 dev/probes/areg_stats_cost.py > $O/areg.jsonl 2> $O/areg.err || { tail -20 $O/areg.err; exit 1; }
cat $O/areg.jsonl
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model resnet50 --no-plain-run --no-extra-configs > $O/r$i.json 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r$i.json'));print('r$i',d['value'],d['ms_per_step'])"
done
echo done
