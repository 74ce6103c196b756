# k_relax time vs the optimality-screen depth and the cut batch (study).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "4 4" "4 0" "4 8" "4 16" "4 64" "8 8" "8 16" "8 64"; do
  set -- $cfg
  SGUFP_SCREEN=$2 timeout -k 10 200 python -u tools/relax_diag.py --cb $1 --nodes 8192 > gpurun_out/screen_cb$1_s$2.log 2>&1 || exit 1
done
