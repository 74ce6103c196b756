# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/calib/calib_fetch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r02}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_calib_fetch -o run -- ./tools/calib/calib_fetch > gpurun_out/${TAG}_calib_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_calib_write -o run -- ./tools/calib/calib_fetch > gpurun_out/${TAG}_calib_write.log 2>&1 && \
python3 tools/calib/calib_table.py gpurun_out/${TAG}_calib_fetch gpurun_out/${TAG}_calib_write > gpurun_out/${TAG}_fetch_calibration.json
