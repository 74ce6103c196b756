#!/bin/bash
# round 4: register groups of the single-wave subproblem kernel (16 = tree, 20 B of scratch at 128
# VGPRs; 14 / 12 none): sub_bench C3 / C4 and the seeded C3 search without the trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for V in tree rg14 rg12; do
  if [ $V = tree ]; then L=sgufp_solver_amd/lib/libsgufp_hip.so; else L=sgufp_solver_amd/lib_var/$V/libsgufp_hip.so; fi
  for A in "C3 26 64" "C4 32 256"; do
    set -- $A
    SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/sub_bench.py --cfg $1 --paths $2 --scenarios $3 --reps 3 \
        > gpurun_out/r04aa_${V}_$1.log 2>&1 || exit $?
    echo "$V $1: $(tail -1 gpurun_out/r04aa_${V}_$1.log)"
  done
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 --no-trace \
      --out gpurun_out/r04aa_$V.json > gpurun_out/r04aa_$V.log 2>&1 || exit $?
  echo "$V $(grep '"total"' gpurun_out/r04aa_$V.log | tail -1)"
done
