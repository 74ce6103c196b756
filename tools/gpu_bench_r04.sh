#!/bin/bash
# round-4 end: kernel stats, HBM (FETCH / WRITE) and issue (SQ) counter passes of the bench
# command, then the bench line itself (which reads the counters back when the library matches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r04
# the profiling passes time the headline step only (the other legs add thousands of launches)
ONLY="--no-cpu --no-parity --sub-paths 0 --c5-nodes 0 --bnb-seeded-width 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-parity-rounds 0"
mkdir -p gpurun_out profiles
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o run -- python3 bench.py --steps 5 --warmup 2 $ONLY > gpurun_out/${TAG}_stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 $ONLY > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 $ONLY > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d gpurun_out/${TAG}_pmc_issue -o run -- python3 bench.py --steps 2 --warmup 1 $ONLY > gpurun_out/${TAG}_pmc_issue.log 2>&1 || exit $?
for d in pmc_fetch pmc_write pmc_issue; do
  sha256sum sgufp_solver_amd/lib/libsgufp_hip.so | cut -d' ' -f1 > gpurun_out/${TAG}_$d/lib.sha256
  python3 tools/kernel_src_sha256.py > gpurun_out/${TAG}_$d/src.sha256
  echo "C4:seed1:nodes8192:pool16F+64O" > gpurun_out/${TAG}_$d/workload.txt
  cp -r gpurun_out/${TAG}_$d profiles/
done
timeout -k 10 900 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
tail -c 600 gpurun_out/bench_${TAG}.json
