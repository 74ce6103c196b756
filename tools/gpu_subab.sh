# Subproblem check + timing in one call: GPU tests of the scenario subproblem, then
# sub_bench on C3 (64 scenarios, 26 paths) and C5 (512 scenarios, 4 paths; the large
# multi-wave variant and, with SGUFP_SUB_WAVES=1, the single-wave one).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subproblem.py -x -v --timeout 300 --timeout-method thread > gpurun_out/sub_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 2 > gpurun_out/sub_c3.log 2>&1 && \
timeout -k 10 200 python -u tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 1 > gpurun_out/sub_c5.log 2>&1 && \
SGUFP_SUB_WAVES=1 timeout -k 10 200 python -u tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 1 > gpurun_out/sub_c5_w1.log 2>&1
