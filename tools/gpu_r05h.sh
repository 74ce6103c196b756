#!/bin/bash
# round 5: non-exact hand-off debug prints (lib_dbg, SGUFP_NX_DEBUG)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_dbg/libsgufp_hip.so timeout -k 10 300 python -u tools/nx_diag.py C4 > gpurun_out/r05h_diag.log 2>&1
rc=$?; grep -E "incumbent|NXDBG" gpurun_out/r05h_diag.log | head -60; exit $rc
