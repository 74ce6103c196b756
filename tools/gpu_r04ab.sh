#!/bin/bash
# round 4: records per B&B round (1 024 vs 2 048) on the seeded C3 search without the trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for B in 1024 2048; do
  timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 --no-trace --batch $B \
      --out gpurun_out/r04ab_$B.json > gpurun_out/r04ab_$B.log 2>&1 || exit $?
  echo "$B $(grep '"total"' gpurun_out/r04ab_$B.log | tail -1)"
done
