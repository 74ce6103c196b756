# Restricted DD parity on the GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_restricted.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/rdd_tests.log 2>&1
