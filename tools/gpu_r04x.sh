#!/bin/bash
# round 4: one packed read-back per refinement iteration: B&B tests, then the seeded C3 search
# without the round trace, previous library (preloop) vs this one
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bnb.py tests/test_bnb_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04x_tests.log; [ $rc -eq 0 ] || exit $rc
for V in preloop tree; do
  if [ $V = tree ]; then L=sgufp_solver_amd/lib/libsgufp_hip.so; else L=sgufp_solver_amd/lib_var/$V/libsgufp_hip.so; fi
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 --no-trace \
      --out gpurun_out/r04x_$V.json > gpurun_out/r04x_$V.log 2>&1 || exit $?
  echo "$V $(grep '"total"' gpurun_out/r04x_$V.log | tail -1)"
done
