# Kernel iteration: DD parity suite (fail fast), then the bench-workload diagnostics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/relax_diag.py --nodes 8192 > gpurun_out/iter_diag.log 2>&1
