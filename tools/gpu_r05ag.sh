#!/bin/bash
# round 5: the unseeded C4 leg at the bench's 20 s, per refinement chunk (variance of the leg vs the 15-s A/B)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in 16384 32768 65536 32768; do
  SGUFP_CHUNK_LPS=$c timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 \
      --nodes 1024 --round-seconds 5 > gpurun_out/r05ag_$c.json 2> gpurun_out/r05ag_$c.err || exit $?
  echo "chunk $c C4 20 s: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05ag_$c.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'], d['rounds'], d['counters']['relaxed'], d['counters']['deferred'], d['counters']['resumed'])")"
done
