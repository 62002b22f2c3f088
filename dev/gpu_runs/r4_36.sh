#!/bin/bash
# ResNet-152 bf16 vs fp8 same-box pair + bf16 kernel breakdown (what an fp8 path could save)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_36
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --model resnet152 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/bf16_$i.json 2> $O/bf16_$i.err || exit $?
  timeout -k 10 240 python3 bench.py --model resnet152 --fp8 --steps 10 --warmup 5 --no-ddp-rehearsal > $O/fp8_$i.json 2> $O/fp8_$i.err || exit $?
done
cat $O/*.json
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d /tmp/r152 -o r152 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet152 --steps 3 --warmup 2 --no-ddp-rehearsal --graph off > $O/prof.log 2>&1 || exit $?
find /tmp/r152 -name "*kernel_trace.csv" -exec cp {} $O/r152_trace.csv \;
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $O/r152_trace.csv --steps 3 --by-grid --top 60 > $O/r152_summary.txt 2>&1
python3 tools/prof_summary.py $O/r152_trace.csv --steps 3 --top 40 > $O/r152_summary_byname.txt 2>&1
head -30 $O/r152_summary_byname.txt | cut -c1-170
