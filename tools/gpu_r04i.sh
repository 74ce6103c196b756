#!/bin/bash
# round 4: lazy terminal weights of exact DDs (SGUFP_EXACT_LAZY): parity with a small cap, C3 B&B at two caps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
SGUFP_EXACT_LAZY=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bnb_parity.py tests/test_bnb.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04i_tests.log; ok $rc || exit $rc
for L in 8 32; do
  SGUFP_EXACT_LAZY=$L SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 \
      --out gpurun_out/r04i_l$L.json > gpurun_out/r04i_l$L.log 2>&1 || exit $?
  echo "lazy $L"; tail -1 gpurun_out/r04i_l$L.log
done
