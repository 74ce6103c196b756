#!/bin/bash
# round 6 final: 2-rank rehearsal of bench.py --gpus 2 on one card (gloo exchanges: RCCL refuses two
# ranks on one device) with the final tree -- the weak-scaled headline step and the bnb_multi leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --nodes 1024 --steps 3 --warmup 1 --no-cpu \
  --sub-paths 0 --bnb-leg-seconds 10 > gpurun_out/r06w_2rank.json 2> gpurun_out/r06w_2rank.err
rc=$?
tail -c 600 gpurun_out/r06w_2rank.json
exit $rc
