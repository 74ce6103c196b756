#!/bin/bash
# round 6: sixteen waves per scenario in the large subproblem kernel (lib_alt/w16,
# -DSGUFP_LARGE_WAVES=16) against eight: C5 4 x 512 cold micro-bench, the C5 B&B (30 s), and the
# subproblem tests on C5 with the variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$PWD/sgufp_solver_amd/lib_alt
for v in tree w16; do
  L=""; [ $v != tree ] && L=$A/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r06v_sub5_$v.log 2>&1 || exit 11
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C5 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-seconds 30 > gpurun_out/r06v_bnb5_$v.json 2> gpurun_out/r06v_bnb5_$v.log || exit 12
done
SGUFP_LIB_PATH=$A/w16/libsgufp_hip.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_subproblem.py -k "C5" > gpurun_out/r06v_tests.log 2>&1
