#!/bin/bash
# round 3: subproblem diagnostics of the dirty-group Bellman-Ford (C1 seed 2, lower bounds 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for env in "SGUFP_SUB_DIRTY=1" "SGUFP_SUB_DIRTY=0" "SGUFP_SUB_KEY64=1"; do
  echo "== $env"
  env $env timeout -k 10 120 python -u tools/sub_debug.py C1 2 1 1 6 || exit 1
done
