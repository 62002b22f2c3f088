#!/bin/bash
# pp FX_STATS epilogue cost: full vs no slab stores vs no sums (variant libraries, tools/pp_one.py traces)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_21
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PDNN_PP_CONV_FWD_K=0 PDNN_PP_CONV_DGRAD_K=0
for V in base noslab nosum; do
  L=""; [ $V != base ] && L=$GRAFT_REPO_ROOT/variants/libpdnn_kernels_$V.so
  for KD in nt fwd1x1; do
    timeout -k 10 60 env ${L:+PDNN_KERNEL_LIB=$L} python -u tools/pp_one.py 802816 256 64 --kind $KD --trace --iters 10 2>&1 | grep -v amdgpu.ids | sed "s/^/$V $KD /" >> $O/trace.log || exit 1
  done
done
echo done
