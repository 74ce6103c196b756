set -o pipefail
mkdir -p gpurun_out
export SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib/variants/prof/libsgufp_hip.so
for cfg in "4 64" "4 40" "8 48"; do set -- $cfg; SGUFP_LDS_KB=$2 timeout -k 10 300 python tools/relax_diag.py --cb $1 > gpurun_out/prof_cb$1_lds$2.log 2>&1 || exit 1; done
