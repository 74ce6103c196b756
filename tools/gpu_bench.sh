# One GPU call: rocprofv3 kernel stats, two PMC passes (HBM bytes), then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_stats.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/${TAG}_pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/${TAG}_pmc_write.log 2>&1 && \
sha256sum sgufp_solver_amd/lib/libsgufp_hip.so | cut -d' ' -f1 > gpurun_out/${TAG}_pmc_fetch/lib.sha256 && \
cp gpurun_out/${TAG}_pmc_fetch/lib.sha256 gpurun_out/${TAG}_pmc_write/lib.sha256 && \
echo "C4:seed1:nodes8192:pool16F+64O" > gpurun_out/${TAG}_pmc_fetch/workload.txt && \
cp gpurun_out/${TAG}_pmc_fetch/workload.txt gpurun_out/${TAG}_pmc_write/workload.txt && \
mkdir -p profiles && cp -r gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write profiles/ && \
timeout -k 10 600 python3 bench.py --profile-tag ${TAG} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
