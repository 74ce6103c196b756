# Traced subproblem (SGUFP_SUB_TRACE variant): augmentations, Bellman-Fords, passes and the
# tick split (Bellman-Ford / walk + augment / predecessors + subtree invalidation) per sampled
# scenario, on C3 (64 scenarios) and C5 (512).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/sgufp_solver_amd/lib_var/trace/libsgufp_hip.so
SGUFP_LIB_PATH=$L timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 0 > gpurun_out/subtr_c3.log 2>&1 && \
SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 0 > gpurun_out/subtr_c5.log 2>&1
