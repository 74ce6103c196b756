#!/bin/bash
# round 6: the non-exact phase's survivors against ref_dd relaxp at 2e4 / 1e5 optimality cuts
# (unseeded C4; the reference sweeps 1e5 cuts per record on the host, a heartbeat keeps
# gpurun_out moving), then the non-exact phase's fixture tests and the C++ host driver
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06m_heartbeat.log; done ) &
HB=$!
timeout -k 10 1000 python3 -u -m pytest -x -v -s --timeout 1500 --timeout-method thread tests/test_bnb_parity.py -k "c4_survivors" \
  > gpurun_out/r06m_survivors.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then kill $HB; exit $rc; fi
timeout -k 10 150 python3 -u -m pytest -x -v --timeout 140 --timeout-method thread tests/test_nx_phase.py tests/test_host_api.py \
  > gpurun_out/r06m_tests.log 2>&1
rc=$?
kill $HB
exit $rc
