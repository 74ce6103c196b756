#!/bin/bash
# round 5: several augmentations per Bellman-Ford in the warm repair (default 16) vs one
# (lib_alt/multi1): warm tests (prod + verify), then the C4 B&B legs with subproblem statistics
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_subproblem.py -k "warm" -v --timeout 240 --timeout-method thread -m gpu \
    > gpurun_out/r05q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05q_tests.log | tail -2; [ $rc -le 1 ] || exit $rc
for v in default multi1; do
  lib=""; [ $v != default ] && lib=$PWD/sgufp_solver_amd/lib_alt/$v/libsgufp_hip.so
  for h in 0 128; do
    SGUFP_LIB_PATH=$lib SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 \
        --nodes 1024 --round-seconds 5 --bnb-heuristic $h > gpurun_out/r05q_${v}_h$h.json 2> gpurun_out/r05q_${v}_h$h.err || exit $?
    echo "$v h=$h: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05q_${v}_h$h.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'])") $(grep '\[sub\]' gpurun_out/r05q_${v}_h$h.err | tail -1)"
  done
done
exit $rc
