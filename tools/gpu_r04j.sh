#!/bin/bash
# round 4: headline k_relax phase split (profiling library) + 4-rank gloo rehearsal of the multi-rank legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_LIB_PATH=sgufp_solver_amd/lib_prof/libsgufp_hip.so timeout -k 10 300 python3 tools/relax_diag.py --config C4 --nodes 8192 \
    > gpurun_out/r04j_relax_phases.log 2>&1 || exit $?
tail -14 gpurun_out/r04j_relax_phases.log
SGUFP_BENCH_BACKEND=gloo timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --nodes 1024 --steps 3 --warmup 1 --no-cpu \
  --sub-paths 0 --bnb-leg-seconds 10 > gpurun_out/r04j_4rank.json 2> gpurun_out/r04j_4rank.err || exit $?
tail -c 1500 gpurun_out/r04j_4rank.json
