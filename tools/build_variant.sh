#!/bin/bash
# Build a libsgufp_hip.so variant with some sources compiled under extra -D flags (A/B studies).
#   tools/build_variant.sh NAME "sub_kernels.hip exact_kernels.hip" -DFLAG=1 ...
# -> sgufp_solver_amd/lib_alt/NAME/libsgufp_hip.so (the other objects as in the tree)
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRCS=$2; shift 2
OUT=sgufp_solver_amd/lib_alt/$NAME
mkdir -p $OUT/obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Isgufp_solver_amd/csrc $*"
for f in dd_kernels.hip sub_kernels.hip bnb_kernels.hip rdd_kernels.hip exact_kernels.hip capi.cpp bnb.cpp network.cpp shard.cpp; do
  if [[ " $SRCS " == *" $f "* ]]; then
    lang=""; [[ $f == *.hip ]] && lang="-x hip"
    /opt/rocm/bin/hipcc $FLAGS $lang -c sgufp_solver_amd/csrc/$f -o $OUT/obj/$f.o
  else
    cp sgufp_solver_amd/lib/obj/$f.o $OUT/obj/$f.o
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsgufp_hip.so $OUT/obj/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $OUT/libsgufp_hip.so
