set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_check.py --cb 1,4,8,16 > gpurun_out/ab.log 2>&1 && \
for cb in 4 8 16; do timeout -k 10 300 python tools/relax_diag.py --cb $cb > gpurun_out/diag_cb$cb.log 2>&1 || exit 1; done
