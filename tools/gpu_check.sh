set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_check.py --cb 1,4,8,16 > gpurun_out/ab.log 2>&1 && \
timeout -k 10 300 python tools/relax_diag.py --cb 4 > gpurun_out/diag_cb4.log 2>&1 && \
timeout -k 10 300 python tools/relax_diag.py --cb 8 > gpurun_out/diag_cb8.log 2>&1
