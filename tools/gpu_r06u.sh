#!/bin/bash
# round 6: the headline step at 8 192 / 12 288 / 16 384 open nodes per launch (DD scratch 114 /
# 171 / 228 GiB of the 288 GB): does a larger resident frontier batch pack the launch better?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ONLY="--no-cpu --no-parity --sub-paths 0 --c5-nodes 0 --bnb-seeded-width 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-parity-rounds 0 --bnb-gen-seconds 0 --cpp-leg-seconds 0 --bnb-parity-survivor-pool 0"
for n in 8192 12288 16384; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --nodes $n $ONLY > gpurun_out/r06u_head_$n.json 2> gpurun_out/r06u_head_$n.log || exit 11
done
