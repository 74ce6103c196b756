#!/bin/bash
# round 5: RelaxedDDNew surface on the device vs the reference (tests/test_dd_api.py), the
# native multi-shard exchanges over the loopback transport (tests/test_native_shards.py), then
# the subproblem paths of the seeded C3 / C4 searches in solve order (warm-start study)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dd_api.py tests/test_native_shards.py -v --timeout 200 \
    --timeout-method thread -m gpu > gpurun_out/r05b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r05b_tests.log
[ $rc -le 1 ] || exit $rc   # a crash / time limit ends the call here
timeout -k 10 200 python -u tools/sub_paths_dump.py --config C3 --seconds 15 --out gpurun_out/r05a_paths_c3.npz > gpurun_out/r05a_c3.log 2>&1 || exit $?
tail -1 gpurun_out/r05a_c3.log
timeout -k 10 200 python -u tools/sub_paths_dump.py --config C4 --width 128 --seconds 15 --out gpurun_out/r05a_paths_c4.npz > gpurun_out/r05a_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r05a_c4.log
exit $rc
