#!/bin/bash
# round 4: leaf-kernel occupancy A/B on the seeded C3 search (grid 4 x CUs, persistent):
# tree = 16 leaves/wave, 64 staged rows, 2 WGs/CU; la = 16 / 40 rows, 3 WGs/CU (80 VGPRs);
# lb = 24 leaves, 2 WGs/CU (128 VGPRs); lc = 8 leaves / 40 rows, 3 WGs/CU (73 VGPRs)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for V in tree la lb lc; do
  if [ $V = tree ]; then L=sgufp_solver_amd/lib/libsgufp_hip.so; else L=sgufp_solver_amd/lib_var/$V/libsgufp_hip.so; fi
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 \
      --out gpurun_out/r04r_$V.json > gpurun_out/r04r_$V.log 2>&1 || exit $?
  echo "$V $(tail -1 gpurun_out/r04r_$V.log)"
done
