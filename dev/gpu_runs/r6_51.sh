#!/bin/bash
# GPT-2 DDP path vs plain step: kernel traces of both (where does the DDP path's ~2% go at N = 1?)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_51
mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/d51 -o d51 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 5 --warmup 3 --no-plain-run --no-extra-configs --diag-steps 0 > $O/ddp.log 2>&1 || exit $?
find /tmp/d51 -name "*kernel_trace.csv" -exec cp {} $O/ddp.csv \;
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/p51 -o p51 --output-format csv -- python3 $R/bench.py --model gpt2_small --steps 5 --warmup 3 --plain --no-extra-configs --diag-steps 0 > $O/plain.log 2>&1 || exit $?
find /tmp/p51 -name "*kernel_trace.csv" -exec cp {} $O/plain.csv \;
cd $R
python3 tools/stream_busy.py $O/ddp.csv --step-kernel adam_kernel --full --top 60 > $O/ddp_streams.txt 2>&1
python3 tools/stream_busy.py $O/plain.csv --step-kernel adam_kernel --full --top 60 > $O/plain_streams.txt 2>&1
head -1 $O/ddp_streams.txt; head -1 $O/plain_streams.txt
echo done
