# relax_diag on library variants (VARS="a b ..."), one log each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARS}; do
  if [ "$v" = base ]; then L=; else L=$PWD/sgufp_solver_amd/lib_var/$v/libsgufp_hip.so; fi
  SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/relax_diag.py --nodes ${NODES:-8192} ${ARGS} > gpurun_out/var_$v.log 2>&1 || exit 1
done
