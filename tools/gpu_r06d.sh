#!/bin/bash
# round 6: closing times of the device B&B on 64-scenario instances between T4 and M1 with the
# generated lower bounds (tools/closure_study.py; HiGHS optima from the CPU study)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python3 -u tools/closure_study.py 100 \
  P1 48 4 6 2 0.45 1 0x1.d4a3c00000000p+12 \
  P1 48 4 6 2 0.45 3 0x1.96c6800000001p+12 \
  P3 52 4 6 2 0.5 2 0x1.0782a00000000p+13 \
  P3 52 4 6 2 0.5 3 0x1.c7e1c00000001p+12 \
  > gpurun_out/r06d_closure.jsonl 2> gpurun_out/r06d_closure.log
