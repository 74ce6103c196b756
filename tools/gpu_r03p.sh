#!/bin/bash
# round 3: early-stop Bellman-Ford (tests + timing), then the device B&B on C3 / C4 with the
# incumbent seeded by the restricted-DD heuristic (incumbent pruning acting, BASELINE configs[2])
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_r03o.sh || exit 1
for c in "C3 64" "C4 128"; do
  set -- $c
  timeout -k 10 200 python3 bench.py --mode bnb --bnb-config $1 --nodes 1024 --bnb-seconds 20 --bnb-heuristic $2 > gpurun_out/r03p_bnb_$1.json 2> gpurun_out/r03p_bnb_$1.err || { tail gpurun_out/r03p_bnb_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03p_bnb_$1.json')); print('$1', d['value'], d['subproblems_per_s'], d['heuristic_incumbent'], d['incumbent'], d['counters'])"
done
