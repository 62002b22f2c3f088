#!/bin/bash
# every GPT-2 GEMM with its epilogue: in-tree tile widths vs hipBLASLt
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_14
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 dev/probes/gpt2_gemms.py > $O/gemms.jsonl 2> $O/gemms.err || { tail -20 $O/gemms.err; exit 1; }
cat $O/gemms.jsonl
