#!/bin/bash
# round 6: open-leaf compaction of the exact leaf passes -- parity (B&B round-by-round checks,
# exact-phase variants, the non-exact phase), then the seeded C4 leg at SGUFP_LEAF_SPLIT
# 0 (one phase) / 8 / 16 (default) / 32, with the exact phase's counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="python3 -u -m pytest -x -v --timeout 400 --timeout-method thread"
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
timeout -k 10 900 $T tests/test_bnb_parity.py -k "c3_seeded or c4 and not survivors and not timed or m1 or variants" tests/test_nx_phase.py \
  > gpurun_out/r06e_tests.log 2>&1 || exit 11
for sp in 16 0 8 32; do
  SGUFP_LEAF_SPLIT=$sp SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06e_bnbs_split$sp.json 2> gpurun_out/r06e_bnbs_split$sp.log || exit 12
done
