#!/bin/bash
# GPT-2 DDP path at the 128 MB bucket default: kernel trace (remaining idle gaps); RCCL-in-graph variant for reference
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_46
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 > $O/ddp.json 2> $O/ddp.err || { tail -20 $O/ddp.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/ddp.json'));print('ddp',d['value'],d['ms_per_step'],d['config'].get('bucket_mb'))"
timeout -k 10 300 python3 bench.py --model gpt2 --no-plain-run --diag-steps 0 --graph collectives > $O/ddp_graph.json 2> $O/ddp_graph.err || { tail -20 $O/ddp_graph.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/ddp_graph.json'));print('ddp graph',d['value'],d['ms_per_step'],d['config'].get('hipgraph'))"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/g12 -o g12 --output-format csv -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 --no-plain-run --diag-steps 0 > $O/g12.log 2>&1 || exit $?
find /tmp/g12 -name "*kernel_trace.csv" -exec cp {} $O/g12_trace.csv \;
echo done
