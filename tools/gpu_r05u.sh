#!/bin/bash
# round 5: Bellman-Ford register-group batching A/B (lib_alt/bfb2, bfb4 vs the tree's lib):
# subproblem micro-bench (C4 32 x 256, C5 4 x 512; digests must agree) and the C4 B&B leg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default bfb2 bfb4; do
  lib=""; [ $v != default ] && lib=$PWD/sgufp_solver_amd/lib_alt/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$lib timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r05u_${v}_c4.log 2>&1 || exit $?
  SGUFP_LIB_PATH=$lib timeout -k 10 120 python3 tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r05u_${v}_c5.log 2>&1 || exit $?
  SGUFP_LIB_PATH=$lib SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 15 \
      --nodes 1024 --round-seconds 5 > gpurun_out/r05u_${v}_bnb.json 2> gpurun_out/r05u_${v}_bnb.err || exit $?
  echo "$v: C4 $(tail -2 gpurun_out/r05u_${v}_c4.log | tr '\n' ' ') | C5 $(tail -2 gpurun_out/r05u_${v}_c5.log | tr '\n' ' ')"
  echo "$v: bnb $(python3 -c "import json;d=json.loads(open('gpurun_out/r05u_${v}_bnb.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'])") $(grep '\[sub\]' gpurun_out/r05u_${v}_bnb.err | tail -1)"
done
