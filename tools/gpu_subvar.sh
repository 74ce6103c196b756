# sub_bench on subproblem library variants (VARS="a b ..."; base = the tree's library).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARS}; do
  if [ "$v" = base ]; then L=; else L=$PWD/sgufp_solver_amd/lib_var/$v/libsgufp_hip.so; fi
  SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/sub_bench.py ${ARGS} > gpurun_out/subvar_$v.log 2>&1 || exit 1
done
