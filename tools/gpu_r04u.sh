#!/bin/bash
# round 4: root folds with prefix checkpoints across sibling records: parity suites, seeded C3
# search (kernel trace), then the round-end bench + counters
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bnb_parity.py tests/test_bnb.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r04u_tests.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04u_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04u_trace -o run -- \
    python3 tools/bnb_tail_diag.py --config C3 --seconds 20 --out gpurun_out/r04u_c3.json > gpurun_out/r04u_c3.log 2>&1 || exit $?
grep '"total"' gpurun_out/r04u_c3.log | tail -1
bash tools/gpu_bench_r04.sh
