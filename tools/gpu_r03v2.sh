#!/bin/bash
# round 3: config-5 relaxation leg at 1024 / 2048 / 4096 records per launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 1024 2048 4096; do
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-parity --sub-paths 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-seeded-width 0 --c5-paths 0 --c5-nodes $n > gpurun_out/r03v2_c5_$n.json 2> gpurun_out/r03v2_c5_$n.err || { tail gpurun_out/r03v2_c5_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03v2_c5_$n.json'))['config5']; print($n, d['relaxations_per_s'], d['k_relax_ms'], d['status_counts'], d['avg_sweeps'])"
done
