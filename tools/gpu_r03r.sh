#!/bin/bash
# round 3: records per B&B round in the seeded device B&B (C3 and C4, 20 s each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in "C3 4096" "C3 8192" "C4 4096" "C4 8192"; do
  set -- $c
  timeout -k 10 240 python3 bench.py --mode bnb --bnb-config $1 --nodes $2 --bnb-seconds 20 --bnb-heuristic 64 > gpurun_out/r03r_$1_$2.json 2> gpurun_out/r03r_$1_$2.err || { tail gpurun_out/r03r_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03r_$1_$2.json')); print('$1 $2', d['value'], d['subproblems_per_s'], d['rounds'], d['counters'])"
done
