# Subproblem iteration: subproblem + B&B GPU tests, then the device B&B bench under a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sub}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --mode bnb --bnb-seconds ${SECS:-20} > gpurun_out/${TAG}_bnb.json 2> gpurun_out/${TAG}_bnb.err
