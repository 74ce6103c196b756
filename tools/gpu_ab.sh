# A/B of subproblem variants built by tools/build_variant.sh (VARS="a b ...")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARS}; do
  SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_var/$v/libsgufp_hip.so timeout -k 10 120 python -u tools/sub_bench.py --reps 2 ${ARGS} > gpurun_out/ab_$v.log 2>&1 || exit 1
done
