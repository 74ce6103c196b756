# Round-end check in one call: GPU suite, smoke, profiled bench (stats + PMC passes + bench
# line), device B&B bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
TAG=r01 bash tools/gpu_bench.sh && \
timeout -k 10 600 python3 bench.py --mode bnb --nodes 1024 --bnb-seconds 20 > gpurun_out/r01_bnb.json 2> gpurun_out/r01_bnb.err
