#!/bin/bash
# Build libsgufp_hip.so variants for A/B timing (study tool).
#   tools/build_variant.sh NAME SUB_KERNELS_SOURCE [extra hipcc flags...]
# -> sgufp_solver_amd/lib_var/NAME/libsgufp_hip.so (every other source as in the tree)
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; shift 2
OUT=sgufp_solver_amd/lib_var/$NAME
mkdir -p $OUT/obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Isgufp_solver_amd/csrc $*"
/opt/rocm/bin/hipcc $FLAGS -x hip -c $SRC -o $OUT/obj/sub.o
for f in dd_kernels.hip bnb_kernels.hip rdd_kernels.hip exact_kernels.hip; do
  cp sgufp_solver_amd/lib/obj/$f.o $OUT/obj/$f.o
done
for f in capi.cpp bnb.cpp network.cpp shard.cpp; do cp sgufp_solver_amd/lib/obj/$f.o $OUT/obj/$f.o; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsgufp_hip.so $OUT/obj/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $OUT/libsgufp_hip.so
