#!/bin/bash
# Build an experimental variant of the library: tools/build_variant.sh NAME 'sed-expr' ...
# -> varlib/NAME.so (load it with DRAGG_LIB=varlib/NAME.so).  Not part of the product.
set -e
NAME=$1; shift
OUTDIR=${OUTDIR:-varlib}
mkdir -p $OUTDIR
SRC=dragg_amd/csrc/_var_$NAME.hip
cp dragg_amd/csrc/mpc_kernel.hip $SRC
for e in "$@"; do sed -i -e "$e" $SRC; done
if [ $# -gt 0 ] && cmp -s dragg_amd/csrc/mpc_kernel.hip $SRC; then echo "variant $NAME: no change"; rm -f $SRC; exit 1; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC \
  -Wno-unused-function -Wno-unused-variable -mllvm -amdgpu-sched-strategy=iterative-ilp \
  -o $OUTDIR/$NAME.so $SRC
rm -f $SRC
echo $OUTDIR/$NAME.so
