#!/bin/bash
# round 5: how many exact-DD leaves stay open past the first cut blocks (leaf-pass compaction?)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_EXACT_STATS=1 timeout -k 10 200 python -u tools/bnb_tail_diag.py --config C3 --seconds 20 --no-trace \
      --width 64 --out gpurun_out/r05m_C3.json > gpurun_out/r05m_C3.log 2>&1 || exit $?
tail -1 gpurun_out/r05m_C3.log | cut -c1-300
grep "exact leaves [1-9]" gpurun_out/r05m_C3.log | awk -F'exact leaves ' '{print $2}' | sort | uniq | tail -40
