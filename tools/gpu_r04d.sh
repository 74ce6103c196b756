#!/bin/bash
# round 4: refinement iterations per round (bnb_set_limits) on the seeded C3 B&B with the
# cut-parallel exact phase; duplicate subproblem paths
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for it in 0 2 4 8 16; do
  timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 25 --round-iters $it \
    --out gpurun_out/r04d_it$it.json > gpurun_out/r04d_it$it.log 2>&1 || exit $?
  tail -1 gpurun_out/r04d_it$it.log
done
