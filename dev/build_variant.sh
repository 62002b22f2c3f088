#!/bin/bash
# A/B kernel library: gemm_mfma.hip rebuilt with extra defines, linked with the other in-tree objects.
# usage: dev/build_variant.sh NAME -DFOO=1 ...   -> dev_lib/libpdnn_kernels_NAME.so (PDNN_KERNEL_LIB=...)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p $R/dev_lib/obj_$N
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -munsafe-fp-atomics -I$R/csrc/include -I$R/csrc/kernels -mllvm -amdgpu-mfma-vgpr-form=1"
/opt/rocm/bin/hipcc $F "$@" -c $R/csrc/kernels/gemm_mfma.hip -o $R/dev_lib/obj_$N/gemm_mfma.o
OBJS=$(ls $R/build/kernels/*.o | grep -v gemm_mfma.o)
/opt/rocm/bin/hipcc $F -shared $R/dev_lib/obj_$N/gemm_mfma.o $OBJS -o $R/dev_lib/libpdnn_kernels_$N.so
echo $R/dev_lib/libpdnn_kernels_$N.so
