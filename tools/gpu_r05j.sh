#!/bin/bash
# round 5: non-exact phase after 256 in-order O cuts, early-stopping leaf passes + maxState
# completion: diagnostics, parity (fixtures, bench workload, B&B at real pool sizes), then the
# seeded C3 / C4 searches with it on and off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/nx_diag.py C4 > gpurun_out/r05j_diag.log 2>&1
rc=$?; grep -E "incumbent|\[exact\]" gpurun_out/r05j_diag.log | head -20; [ $rc -eq 0 ] || exit $rc
SGUFP_EXACT_STATS=1 timeout -k 10 1100 python -u -m pytest tests/test_nx_phase.py tests/test_bnb_parity.py -v --timeout 600 \
    --timeout-method thread -m gpu > gpurun_out/r05j_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "passed|failed" gpurun_out/r05j_parity.log | tail -2
grep -E "FAILED" gpurun_out/r05j_parity.log | head -10
[ $rc -le 1 ] || exit $rc
for nx in 1 0; do
  for c in C3 C4; do
    SGUFP_NX=$nx timeout -k 10 200 python -u tools/bnb_tail_diag.py --config $c --seconds 20 --no-trace \
        --width $([ $c = C3 ] && echo 64 || echo 128) --out gpurun_out/r05j_${c}_nx$nx.json > gpurun_out/r05j_${c}_nx$nx.log 2>&1 || exit $?
    echo "$c nx=$nx: $(tail -1 gpurun_out/r05j_${c}_nx$nx.log | cut -c1-300)"
  done
done
exit $rc
