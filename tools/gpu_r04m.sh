#!/bin/bash
# round 4: 8-byte chain records in the single-wave subproblem kernel only: tests, sub_bench, seeded B&B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_subproblem.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/r04m_tests.log 2>&1
rc=$?; echo "sub tests rc=$rc"; tail -2 gpurun_out/r04m_tests.log; [ $rc -eq 0 ] || exit $rc
for A in "C3 26 64" "C4 32 256" "C5 4 512"; do
  set -- $A
  timeout -k 10 200 python3 tools/sub_bench.py --cfg $1 --paths $2 --scenarios $3 --reps 3 > gpurun_out/r04m_$1.log 2>&1 || exit $?
  echo "$1: $(tail -1 gpurun_out/r04m_$1.log)"
done
for C in C3; do
  timeout -k 10 200 python3 tools/bnb_tail_diag.py --config $C --seconds 20 \
      --width $([ $C = C3 ] && echo 64 || echo 128) --out gpurun_out/r04m_bnb_$C.json > gpurun_out/r04m_bnb_$C.log 2>&1 || exit $?
  echo "$C"; tail -1 gpurun_out/r04m_bnb_$C.log
done
