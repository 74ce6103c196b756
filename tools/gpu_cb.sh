# k_relax timing at cut batch sizes 4 / 8 / 16 (SGUFP_CUT_BATCH) on the bench workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cb in 4 8 16; do
  timeout -k 10 200 python -u tools/relax_diag.py --cb $cb --nodes 8192 > gpurun_out/cb_$cb.log 2>&1 || exit 1
done
