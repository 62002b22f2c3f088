#!/bin/bash
# ResNet-152 fp8 kernel breakdown (the fp8 halo conv in the step) + same-box bf16 / fp8 pair
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_40
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cut -c1-200 $O/*.json
timeout -k 10 120 python3 dev/probes/c3_fp8.py > $O/c3_fp8.jsonl 2>&1 || exit $?
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d /tmp/r152f -o r152f --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet152 --fp8 --steps 3 --warmup 2 --no-ddp-rehearsal --graph off > $O/prof.log 2>&1 || exit $?
find /tmp/r152f -name "*kernel_trace.csv" -exec cp {} $O/r152f_trace.csv \;
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $O/r152f_trace.csv --steps 3 --top 40 > $O/r152f_summary_byname.txt 2>&1
head -25 $O/r152f_summary_byname.txt | cut -c1-150
