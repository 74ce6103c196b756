#!/bin/bash
# round 5: warm starts (source re-seeding fix) and the cut-parallel optimality phase of
# non-exact DDs -- parity first, then the seeded C3 / C4 B&B with it on and off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tests/helpers/sub_run.py C3 4 8 12 gpurun_out/r05f_c3.npz warm > gpurun_out/r05f_diag.log 2>&1 || exit $?
python - <<'PY'
import numpy as np
r = np.load("gpurun_out/r05f_c3.npz")
a = r["warm_aug"].ravel(); cold = r["cold_aug"].ravel(); neg = a[a < 0]
print("c3 warm mean", a[a >= 0].mean() if (a >= 0).any() else None, "cold mean", cold.mean(), "fallbacks", len(neg), "of", len(a),
      "why", np.unique((-neg - 1) // 100000, return_counts=True))
PY
timeout -k 10 900 python -u -m pytest tests/test_nx_phase.py tests/test_subproblem.py -k "nx or warm" -v --timeout 300 \
    --timeout-method thread -m gpu > gpurun_out/r05f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05f_tests.log | tail -2
grep -E "FAILED" gpurun_out/r05f_tests.log | head -10
[ $rc -le 1 ] || exit $rc
for nx in 1 0; do
  for c in C3 C4; do
    SGUFP_NX=$nx timeout -k 10 200 python -u tools/bnb_tail_diag.py --config $c --seconds 20 --no-trace \
        --width $([ $c = C3 ] && echo 64 || echo 128) --out gpurun_out/r05f_${c}_nx$nx.json > gpurun_out/r05f_${c}_nx$nx.log 2>&1 || exit $?
    echo "$c nx=$nx: $(tail -1 gpurun_out/r05f_${c}_nx$nx.log | cut -c1-300)"
  done
done
exit $rc
