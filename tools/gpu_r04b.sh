#!/bin/bash
# round 4: the bench line with its new legs (all-core CPU baseline, bnb_parity), then a
# 2-rank gloo rehearsal of the multi-rank legs (weak-scaling DD step + the shared B&B search)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py --profile-tag r03 > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || exit $?
SGUFP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --nodes 1024 --steps 3 --warmup 1 --no-cpu \
  --sub-paths 0 --bnb-leg-seconds 10 > gpurun_out/r04b_2rank.json 2> gpurun_out/r04b_2rank.err
