#!/bin/bash
# round 6: the C++ host driver against the Python one at scale (unseeded C3, 60 rounds); then the
# closing times of the device B&B on the 64-scenario P1 / P3 instances (generated lower bounds,
# tools/closure_study.py; HiGHS optima of tests/golden/extensive_form.json), seeded opt - 10 and
# unseeded, 90 s each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 220 --timeout-method thread tests/test_host_api.py -k "at_scale" \
  > gpurun_out/r06r_host.log 2>&1
timeout -k 10 900 python3 -u tools/closure_study.py 90 \
  P1 48 4 6 2 0.45 1 0x1.d4a3c00000000p+12 \
  P1 48 4 6 2 0.45 3 0x1.96c6800000001p+12 \
  P3 52 4 6 2 0.5 2 0x1.0782a00000000p+13 \
  P3 52 4 6 2 0.5 3 0x1.c7e1c00000001p+12 \
  > gpurun_out/r06r_closure.jsonl 2> gpurun_out/r06r_closure.log
