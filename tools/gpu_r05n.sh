#!/bin/bash
# round 5: exact-leaf pass variants on the seeded C3 / C4 searches (20 s each):
# default (ancestors in registers, 6 waves/SIMD bound), mw5 (registers, 5 waves/SIMD), lds (walk_down)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default mw5 lds; do
  lib=""; [ $v != default ] && lib=$PWD/sgufp_solver_amd/lib_alt/$v/libsgufp_hip.so
  for c in C3 C4; do
    SGUFP_LIB_PATH=$lib timeout -k 10 200 python -u tools/bnb_tail_diag.py --config $c --seconds 20 --no-trace \
        --width $([ $c = C3 ] && echo 64 || echo 128) --out gpurun_out/r05n_${c}_$v.json > gpurun_out/r05n_${c}_$v.log 2>&1 || exit $?
    echo "$c $v: $(tail -1 gpurun_out/r05n_${c}_$v.log | cut -c1-260)"
  done
done
