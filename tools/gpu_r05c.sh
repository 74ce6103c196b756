#!/bin/bash
# round 5: warm-started subproblems -- correctness (warm vs cold, verify build), RelaxedDDNew
# after the dd_bind fix, then the seeded C3 / C4 B&B with and without warm starts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_subproblem.py tests/test_dd_api.py -v --timeout 240 \
    --timeout-method thread -m gpu > gpurun_out/r05c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05c_tests.log | tail -2
[ $rc -le 1 ] || exit $rc
for w in 1 0; do
  for c in C3 C4; do
    SGUFP_SUB_WARM=$w timeout -k 10 200 python -u tools/bnb_tail_diag.py --config $c --seconds 20 --no-trace \
        --width $([ $c = C3 ] && echo 64 || echo 128) --out gpurun_out/r05c_${c}_w$w.json > gpurun_out/r05c_${c}_w$w.log 2>&1 || exit $?
    echo "$c warm=$w: $(tail -1 gpurun_out/r05c_${c}_w$w.log | cut -c1-300)"
  done
done
exit $rc
