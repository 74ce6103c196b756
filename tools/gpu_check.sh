set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_subproblem.py -x -q -m gpu > gpurun_out/sub.log 2>&1
