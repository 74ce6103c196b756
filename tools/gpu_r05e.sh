#!/bin/bash
# round 5: warm-start repair diagnostics (debug build prints the state of an unreachable target)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_dbg/libsgufp_hip.so timeout -k 10 200 python -u tests/helpers/sub_run.py C3 4 8 12 gpurun_out/r05e_c3.npz warm > gpurun_out/r05e_diag.log 2>&1
rc=$?; grep WARMDBG gpurun_out/r05e_diag.log | head -30; exit $rc
