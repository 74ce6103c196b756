#!/bin/bash
# round 5: warm starts after the imbalance-layout fix -- the reasons of any fallback, the warm
# tests, then the seeded C3 / C4 B&B with and without warm starts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tests/helpers/sub_run.py C3 4 8 12 gpurun_out/r05d_c3.npz warm > gpurun_out/r05d_diag.log 2>&1 || exit $?
timeout -k 10 200 python -u tests/helpers/sub_run.py C4 1 256 4 gpurun_out/r05d_c4.npz warm >> gpurun_out/r05d_diag.log 2>&1 || exit $?
python - <<'PY'
import numpy as np
for c in ("c3", "c4"):
    r = np.load(f"gpurun_out/r05d_{c}.npz")
    a = r["warm_aug"].ravel(); cold = r["cold_aug"].ravel()
    neg = a[a < 0]
    print(c, "warm mean", a[a >= 0].mean() if (a >= 0).any() else None, "cold mean", cold.mean(),
          "fallbacks", len(neg), "of", len(a), "why", np.unique((-neg - 1) // 100000, return_counts=True))
PY
timeout -k 10 600 python -u -m pytest tests/test_subproblem.py -k "warm" -v --timeout 240 \
    --timeout-method thread -m gpu > gpurun_out/r05d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05d_tests.log | tail -2
[ $rc -le 1 ] || exit $rc
for w in 1 0; do
  for c in C3 C4; do
    SGUFP_SUB_WARM=$w timeout -k 10 200 python -u tools/bnb_tail_diag.py --config $c --seconds 20 --no-trace \
        --width $([ $c = C3 ] && echo 64 || echo 128) --out gpurun_out/r05d_${c}_w$w.json > gpurun_out/r05d_${c}_w$w.log 2>&1 || exit $?
    echo "$c warm=$w: $(tail -1 gpurun_out/r05d_${c}_w$w.log | cut -c1-300)"
  done
done
exit $rc
