#!/bin/bash
# pp engine phase traces + ablations on short-K shapes (ResNet 1x1 expansions) and a GPT-2 shape
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_19
mkdir -p $O
cd $GRAFT_REPO_ROOT
for S in "802816 256 64" "200704 512 128" "50176 1024 256" "8192 3072 768"; do
  timeout -k 10 60 python -u tools/pp_one.py $S --trace --iters 10 >> $O/trace.log 2>&1 || exit 1
  for A in 1 2 3 4 7; do
    timeout -k 10 60 env PDNN_PP_ABLATE=$A python -u tools/pp_one.py $S --bn 256 --iters 10 2>&1 | sed "s/^/abl$A /" >> $O/trace.log || exit 1
  done
done
echo done
