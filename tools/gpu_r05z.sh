#!/bin/bash
# round 5: LDS cut row vs the HBM atomics (lib_alt/nolacc) on the failing subproblem case
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default nolacc; do
  lib=""; [ $v != default ] && lib=$PWD/sgufp_solver_amd/lib_alt/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$lib timeout -k 10 200 python -u -m pytest tests/test_subproblem.py -q --timeout 120 --timeout-method thread -m gpu \
      -k "matches_highs or benchmark_scenario" > gpurun_out/r05z_$v.log 2>&1
  echo "$v rc=$?: $(tail -1 gpurun_out/r05z_$v.log)"; grep FAILED gpurun_out/r05z_$v.log | head -5
done
for v in default nolacc; do
  lib=""; [ $v != default ] && lib=$PWD/sgufp_solver_amd/lib_alt/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$lib timeout -k 10 100 python3 tools/sub_bench.py --cfg C3 --scenarios 4 --paths 3 --reps 1 > gpurun_out/r05z_sb_$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/r05z_sb_$v.log)"
done
