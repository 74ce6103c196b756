#!/bin/bash
# round 4: cut batch 8 vs 4 in the seeded C3 search (1 024-record rounds fill half the wave slots)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for CB in 4 8; do
  SGUFP_CUT_BATCH=$CB timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 26 \
      --out gpurun_out/r04v_cb$CB.json > gpurun_out/r04v_cb$CB.log 2>&1 || exit $?
  echo "cb $CB $(grep '"total"' gpurun_out/r04v_cb$CB.log | tail -1)"
done
