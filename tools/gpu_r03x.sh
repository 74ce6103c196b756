#!/bin/bash
# round 3: several frontier shards per device (one context / stream / host thread each) in the
# seeded device B&B: 1 / 2 / 4 shards on C3 and C4, 20 s each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in "C3 64" "C4 128"; do
  set -- $c
  for s in 1 2 4; do
    timeout -k 10 200 python3 bench.py --mode bnb --bnb-config $1 --nodes 1024 --bnb-seconds 20 --bnb-heuristic $2 --bnb-streams $s > gpurun_out/r03x_$1_s$s.json 2> gpurun_out/r03x_$1_s$s.err || { tail gpurun_out/r03x_$1_s$s.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03x_$1_s$s.json')); c=d['counters']; print('$1 streams $s', d['value'], d['subproblems_per_s'], d['incumbent'], c['pruned_optimality'], c['exact'], c['resumed'])"
  done
done
