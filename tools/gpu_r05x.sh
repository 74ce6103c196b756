#!/bin/bash
# round 5: repair from zero potentials for paths without a warm source (SGUFP_SUB_ZERO_WARM=1)
# vs the cold SSP: subproblem tests under the flag, micro-bench C4 / C5, C4 / C5 B&B legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_SUB_ZERO_WARM=1 timeout -k 10 400 python -u -m pytest tests/test_subproblem.py -x -q --timeout 240 --timeout-method thread -m gpu \
    > gpurun_out/r05x_tests.log 2>&1
rc=$?; echo "tests(zero warm) rc=$rc"; tail -2 gpurun_out/r05x_tests.log; [ $rc -eq 0 ] || exit $rc
for z in 0 1; do
  export SGUFP_SUB_ZERO_WARM=$z
  timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r05x_z${z}_c4.log 2>&1 || exit $?
  timeout -k 10 150 python3 tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r05x_z${z}_c5.log 2>&1 || exit $?
  echo "z=$z: C4 $(tail -2 gpurun_out/r05x_z${z}_c4.log | head -1) | C5 $(tail -2 gpurun_out/r05x_z${z}_c5.log | head -1)"
  for c in C4 C5; do
    SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config $c --bnb-lb zero --bnb-seconds 15 \
        --nodes 1024 --round-seconds 5 > gpurun_out/r05x_z${z}_$c.json 2> gpurun_out/r05x_z${z}_$c.err || exit $?
    echo "z=$z $c bnb: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05x_z${z}_$c.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'])") $(grep '\[sub\]' gpurun_out/r05x_z${z}_$c.err | tail -1)"
  done
done
