#!/bin/bash
# round 5: the C5 B&B leg (30 s, as the bench runs it) at 16384 / 32768 / 65536 scenario LPs per refinement iteration
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in 16384 32768 65536; do
  SGUFP_CHUNK_LPS=$c timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C5 --bnb-lb zero --bnb-seconds 30 \
      --nodes 1024 --round-seconds 5 > gpurun_out/r05ad_$c.json 2> gpurun_out/r05ad_$c.err || exit $?
  echo "chunk $c C5: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05ad_$c.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'], d['rounds'], d['counters']['deferred'], d['counters']['resumed'])")"
done
