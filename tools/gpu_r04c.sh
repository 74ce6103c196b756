#!/bin/bash
# round 4: the cut-parallel optimality phase of exact DDs (exact_kernels.hip): parity suites,
# then the seeded C3 B&B with it off / on (per-round k_relax time, tail)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bnb.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04c_tests.log 2>&1
rc=$?; echo "parity+bnb rc=$rc"; tail -3 gpurun_out/r04c_tests.log; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_bnb_parity.py -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/r04c_bnbpar.log 2>&1
rc=$?; echo "bnb parity rc=$rc"; tail -3 gpurun_out/r04c_bnbpar.log; ok $rc || exit $rc
for f in 0 1; do
  SGUFP_EXACT_FAST=$f SGUFP_LIB_PATH=sgufp_solver_amd/lib_prof/libsgufp_hip.so timeout -k 10 200 python3 tools/bnb_tail_diag.py \
    --config C3 --seconds 25 --out gpurun_out/r04c_tail_f$f.json > gpurun_out/r04c_tail_f$f.log 2>&1 || exit $?
  tail -1 gpurun_out/r04c_tail_f$f.log
done
