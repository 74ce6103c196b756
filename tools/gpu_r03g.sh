#!/bin/bash
# round 3: rehearse the multi-rank bench (2 ranks on the one card, gloo exchanges) and the
# multi-rank B&B leg protocol
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export SGUFP_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --nodes 2048 > gpurun_out/r03g_bench2.json 2> gpurun_out/r03g_bench2.err || { tail -30 gpurun_out/r03g_bench2.err; exit 1; }
cat gpurun_out/r03g_bench2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --mode bnb --gpus 2 --bnb-config C3 --nodes 256 --bnb-seconds 15 > gpurun_out/r03g_bnb2.json 2> gpurun_out/r03g_bnb2.err || { tail -30 gpurun_out/r03g_bnb2.err; exit 1; }
cat gpurun_out/r03g_bnb2.json
