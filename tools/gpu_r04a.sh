#!/bin/bash
# round 4: device-B&B parity under real Benders pools (tests/test_bnb_parity.py), the
# B&B tests, and the C3 fixture dump for tests/golden/make_bnb_golden.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # test failures go on, faults / timeouts stop
timeout -k 10 300 python -u tools/dump_bnb_fixture.py --config C3 --seed 1 --width 64 --rounds 3 \
    --out gpurun_out/bnb_c3_seeded > gpurun_out/r04a_dump.log 2>&1
rc=$?; echo "dump rc=$rc"; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_bnb_parity.py -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/r04a_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -5 gpurun_out/r04a_parity.log; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_bnb.py -x -v -k "tiny" --timeout 300 --timeout-method thread \
    > gpurun_out/r04a_bnb.log 2>&1
rc=$?; echo "bnb rc=$rc"; tail -3 gpurun_out/r04a_bnb.log
exit $rc
