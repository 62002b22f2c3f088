#!/bin/bash
# pp engine: fused 1x1 conv epilogues traced against the plain GEMM of the same shape; whole-step bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_20
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.log 2>&1 && tail -n 1 $O/bench_default.log
timeout -k 10 200 env PDNN_PP_CONV_MINN=100000 python -u bench.py --steps 20 --warmup 5 > $O/bench_nopp.log 2>&1 && tail -n 1 $O/bench_nopp.log
export PDNN_PP_CONV_FWD_K=0 PDNN_PP_CONV_DGRAD_K=0
for S in "802816 256 64" "200704 512 128"; do
  for KD in nt fwd1x1 fwd1x1pro; do
    timeout -k 10 60 python -u tools/pp_one.py $S --kind $KD --trace --iters 10 2>&1 | sed "s/^/$KD /" >> $O/trace.log || exit 1
  done
done
for S in "200704 128 512" "50176 256 1024"; do
  for KD in nn dgrad1x1bn; do
    timeout -k 10 60 python -u tools/pp_one.py $S --kind $KD --trace --iters 10 2>&1 | sed "s/^/$KD /" >> $O/trace.log || exit 1
  done
done
echo done
