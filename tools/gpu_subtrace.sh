# Traced subproblem (SGUFP_SUB_TRACE variant): augmentations, extra paths, Bellman-Fords,
# passes and tick split per sampled wave, single-path vs multi-path phases.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/sgufp_solver_amd/lib_var/trace/libsgufp_hip.so
for mm in ${MODES:-0 1}; do
  SGUFP_LIB_PATH=$L SGUFP_SUB_MULTI=$mm timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 0 > gpurun_out/subtr_c3_m$mm.log 2>&1 || exit 1
  SGUFP_LIB_PATH=$L SGUFP_SUB_MULTI=$mm timeout -k 10 200 python -u tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 0 > gpurun_out/subtr_c5_m$mm.log 2>&1 || exit 1
done
