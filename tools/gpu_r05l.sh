#!/bin/bash
# round 5: the survivors' large-pool parity (C3) and the seeded C3 search's kernel times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_EXACT_STATS=1 timeout -k 10 900 python -u -m pytest tests/test_bnb_parity.py -k "survivors or timed_pool" -v --timeout 800 \
    --timeout-method thread -m gpu > gpurun_out/r05l_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "passed|failed" gpurun_out/r05l_parity.log | tail -2
grep -E "FAILED|^E " gpurun_out/r05l_parity.log | head -6 | cut -c1-600
[ $rc -le 1 ] || exit $rc
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05l_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/bnb_tail_diag.py" --config C3 --seconds 20 --no-trace --width 64 \
    --out "$GRAFT_REPO_ROOT/gpurun_out/r05l_prof_c3.json" > "$GRAFT_REPO_ROOT/gpurun_out/r05l_prof.log" 2>&1
rc2=$?; cd "$GRAFT_REPO_ROOT"; f=$(ls gpurun_out/r05l_prof/*kernel_stats.csv gpurun_out/r05l_prof/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && head -16 "$f" | cut -c1-220
exit $(( rc > 1 ? rc : rc2 ))
