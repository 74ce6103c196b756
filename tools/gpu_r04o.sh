#!/bin/bash
# round 4: leaf-kernel sizing A/B on the seeded C3 search (tree = 16 layers / 64 rows / 32 leaves
# per wave at 2 waves per SIMD; v8 = 8 / 40; v8h = + 16 leaves, 4 waves per SIMD; v8q = 8 / 40 /
# 32 leaves, 4 waves per SIMD)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for V in tree v8 v8h v8q; do
  if [ $V = tree ]; then L=sgufp_solver_amd/lib/libsgufp_hip.so; else L=sgufp_solver_amd/lib_var/$V/libsgufp_hip.so; fi
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 \
      --out gpurun_out/r04o_$V.json > gpurun_out/r04o_$V.log 2>&1 || exit $?
  echo "$V $(tail -1 gpurun_out/r04o_$V.log)"
done
