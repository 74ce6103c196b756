#!/bin/bash
# round 3: four-rank rehearsal of the weak-scaling bench on one card (gloo exchanges; RCCL
# refuses several ranks per device): the per-step incumbent all-reduce + cut all-gather path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export SGUFP_BENCH_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 4 --steps 5 --warmup 2 --nodes 2048 > gpurun_out/r03w_bench4.json 2> gpurun_out/r03w_bench4.err || { tail -30 gpurun_out/r03w_bench4.err; exit 1; }
cat gpurun_out/r03w_bench4.json
