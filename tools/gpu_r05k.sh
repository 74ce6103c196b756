#!/bin/bash
# round 5: how many records the non-exact phase takes in the seeded B&B, and what it costs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in C3 C4; do
  SGUFP_EXACT_STATS=1 timeout -k 10 200 python -u tools/bnb_tail_diag.py --config $c --seconds 20 --no-trace \
      --width $([ $c = C3 ] && echo 64 || echo 128) --out gpurun_out/r05k_${c}_nx1.json > gpurun_out/r05k_${c}_nx1.log 2>&1 || exit $?
  echo "$c nx=1: $(tail -1 gpurun_out/r05k_${c}_nx1.log | cut -c1-300)"
  grep "handed off [1-9]" gpurun_out/r05k_${c}_nx1.log | tail -4 | cut -c1-330
  echo "launches with hand-offs: $(grep -c 'handed off [1-9]' gpurun_out/r05k_${c}_nx1.log) of $(grep -c 'handed off' gpurun_out/r05k_${c}_nx1.log)"
done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r05k_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/bnb_tail_diag.py" --config C3 --seconds 15 --no-trace --width 64 \
    --out "$GRAFT_REPO_ROOT/gpurun_out/r05k_prof_c3.json" > "$GRAFT_REPO_ROOT/gpurun_out/r05k_prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; f=$(ls gpurun_out/r05k_prof/*/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -14 "$f" | cut -c1-200
exit $rc
