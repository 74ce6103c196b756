#!/bin/bash
# Build a libsgufp_hip.so variant with k_relax / the exact kernels compiled under extra -D flags
# (A/B timing of the leaf-kernel sizing; study tool).
#   tools/build_leaf_variant.sh NAME -DSGUFP_EXACT_MAXT=8 ...
# -> sgufp_solver_amd/lib_alt/NAME/libsgufp_hip.so (the other objects as in the tree)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
OUT=sgufp_solver_amd/lib_alt/$NAME
mkdir -p $OUT/obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Isgufp_solver_amd/csrc $*"
for f in dd_kernels.hip exact_kernels.hip; do
  /opt/rocm/bin/hipcc $FLAGS -x hip -c sgufp_solver_amd/csrc/$f -o $OUT/obj/$f.o
done
for f in sub_kernels.hip bnb_kernels.hip rdd_kernels.hip capi.cpp bnb.cpp network.cpp shard.cpp; do
  cp sgufp_solver_amd/lib/obj/$f.o $OUT/obj/$f.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsgufp_hip.so $OUT/obj/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $OUT/libsgufp_hip.so
