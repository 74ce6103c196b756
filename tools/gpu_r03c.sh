#!/bin/bash
# round 3: GPU suite + smoke, then the profiled bench: kernel stats, PMC passes (HBM bytes,
# issue counters), the bench line reading this build's PMC bytes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r03}
mkdir -p gpurun_out profiles
LEGS="--bnb-leg-seconds 0 --c5-nodes 0 --sub-paths 0 --no-cpu"
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 170 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o run -- python3 bench.py --steps 5 --warmup 2 $LEGS > gpurun_out/${TAG}_stats.log 2>&1 || { tail gpurun_out/${TAG}_stats.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 $LEGS > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { tail gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 $LEGS > gpurun_out/${TAG}_pmc_write.log 2>&1 || { tail gpurun_out/${TAG}_pmc_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/${TAG}_pmc_issue -o run -- python3 bench.py --steps 2 --warmup 1 $LEGS > gpurun_out/${TAG}_pmc_issue.log 2>&1 || { tail gpurun_out/${TAG}_pmc_issue.log; exit 1; }
sha256sum sgufp_solver_amd/lib/libsgufp_hip.so | cut -d' ' -f1 > gpurun_out/${TAG}_pmc_fetch/lib.sha256
python3 tools/kernel_src_sha256.py > gpurun_out/${TAG}_pmc_fetch/src.sha256
for d in pmc_write pmc_issue; do cp gpurun_out/${TAG}_pmc_fetch/lib.sha256 gpurun_out/${TAG}_pmc_fetch/src.sha256 gpurun_out/${TAG}_$d/; done
for d in pmc_fetch pmc_write pmc_issue; do echo "C4:seed1:nodes8192:pool16F+64O" > gpurun_out/${TAG}_$d/workload.txt; cp -r gpurun_out/${TAG}_$d profiles/; done
timeout -k 10 900 python3 bench.py --profile-tag ${TAG} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
