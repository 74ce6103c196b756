# Full GPU suite + smoke + device B&B bench (one call).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py --mode bnb --bnb-seconds ${SECS:-30} > gpurun_out/bnb_bench.json 2> gpurun_out/bnb_bench.err
