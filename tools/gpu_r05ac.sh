#!/bin/bash
# round 5: scenario LPs per refinement iteration (SGUFP_CHUNK_LPS) now that warm scenarios are cheap
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in 16384 32768 65536; do
  for leg in "C4 0" "C4 128" "C3 64"; do
    set -- $leg
    SGUFP_CHUNK_LPS=$c timeout -k 10 200 python3 bench.py --mode bnb --bnb-config $1 --bnb-lb zero --bnb-seconds 15 \
        --nodes 1024 --round-seconds 5 --bnb-heuristic $2 > gpurun_out/r05ac_${c}_$1_$2.json 2> gpurun_out/r05ac_${c}_$1_$2.err || exit $?
    echo "chunk $c $1 h=$2: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05ac_${c}_$1_$2.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'], d['rounds'], d['counters']['deferred'])")"
  done
done
