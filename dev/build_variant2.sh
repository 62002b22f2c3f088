#!/bin/bash
# A/B kernel library: ONE source file rebuilt with extra defines, linked with the other in-tree objects.
# usage: dev/build_variant2.sh NAME SOURCE.hip -DFOO=1 ...   -> dev_lib/libpdnn_kernels_NAME.so (PDNN_KERNEL_LIB=...)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
SRC=$1; shift
B=$(basename $SRC .hip)
mkdir -p $R/dev_lib/obj_$N
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -munsafe-fp-atomics -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-but-set-variable -Werror=return-type -I$R/csrc/include -I$R/csrc/kernels"
/opt/rocm/bin/hipcc $F "$@" -c -x hip $R/csrc/kernels/$B.hip -o $R/dev_lib/obj_$N/$B.o
OBJS=$(ls $R/build/kernels/*.o | grep -v "/$B.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $R/dev_lib/obj_$N/$B.o $OBJS -o $R/dev_lib/libpdnn_kernels_$N.so
echo $R/dev_lib/libpdnn_kernels_$N.so
