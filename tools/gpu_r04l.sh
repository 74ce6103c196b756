#!/bin/bash
# round 4: 8-byte chain records (32-bit keys) in k_sub_scenario: tests, then A/B vs the round-3
# kernel (base) and the packed kernel at 3 waves/SIMD (p3)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_subproblem.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/r04l_tests.log 2>&1
rc=$?; echo "sub tests rc=$rc"; tail -2 gpurun_out/r04l_tests.log; [ $rc -eq 0 ] || exit $rc
for V in tree base p3; do
  if [ $V = tree ]; then L=sgufp_solver_amd/lib/libsgufp_hip.so; else L=sgufp_solver_amd/lib_var/$V/libsgufp_hip.so; fi
  for A in "C3 26 64" "C4 32 256" "C5 4 512"; do
    set -- $A
    SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/sub_bench.py --cfg $1 --paths $2 --scenarios $3 --reps 3 \
        > gpurun_out/r04l_${V}_$1.log 2>&1 || exit $?
    echo "$V $1: $(tail -1 gpurun_out/r04l_${V}_$1.log)"
  done
done
