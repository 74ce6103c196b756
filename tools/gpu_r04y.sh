#!/bin/bash
# round 4 final: seeded C4 search without the trace, and the 2-rank gloo rehearsal of the bench legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C4 --width 128 --seconds 20 --no-trace \
    --out gpurun_out/r04y_c4.json > gpurun_out/r04y_c4.log 2>&1 || exit $?
grep '"total"' gpurun_out/r04y_c4.log | tail -1
SGUFP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --nodes 1024 --steps 3 --warmup 1 --no-cpu \
  --sub-paths 0 --bnb-leg-seconds 10 > gpurun_out/r04y_2rank.json 2> gpurun_out/r04y_2rank.err || exit $?
tail -c 400 gpurun_out/r04y_2rank.json
