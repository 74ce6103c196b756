#!/bin/bash
# round 6: lower-bound warm-start tests; the B&B with the generated lower bounds (seeded /
# unseeded, subproblem statistics); the non-exact phase on the headline step (A/B); the seeded
# C4 leg with the exact phase's counters; leaf-kernel A/B (used-row staging vs all rows vs
# 5 waves per SIMD).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
ONLY="--no-cpu --no-parity --sub-paths 0 --c5-nodes 0 --bnb-seeded-width 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-parity-rounds 0 --bnb-gen-seconds 0 --cpp-leg-seconds 0 --bnb-parity-survivor-pool 0"
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
timeout -k 10 600 $T tests/test_subproblem.py -k "lower_bounds" > gpurun_out/r06c_tests.log 2>&1 || exit 11
SGUFP_SUB_STATS=1 timeout -k 10 300 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb gen --nodes 1024 --round-seconds 5 \
  --bnb-heuristic 128 --bnb-seconds 20 > gpurun_out/r06c_bnb_gen_seeded.json 2> gpurun_out/r06c_bnb_gen_seeded.log || exit 12
SGUFP_SUB_STATS=1 timeout -k 10 300 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb gen --nodes 1024 --round-seconds 5 \
  --bnb-seconds 20 > gpurun_out/r06c_bnb_gen.json 2> gpurun_out/r06c_bnb_gen.log || exit 13
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $ONLY > gpurun_out/r06c_head_default.json 2> gpurun_out/r06c_head_default.log || exit 14
for skip in 0 8 16; do
  SGUFP_NX_MIN=1 SGUFP_NX_SKIP=$skip timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $ONLY > gpurun_out/r06c_head_nx$skip.json 2> gpurun_out/r06c_head_nx$skip.log || exit 15
done
SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06c_bnbs_estats.json 2> gpurun_out/r06c_bnbs_estats.log || exit 16
for v in allrows w5; do
  SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/$v/libsgufp_hip.so timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06c_bnbs_$v.json 2> gpurun_out/r06c_bnbs_$v.log || exit 17
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06c_bnbs_stats -o run -- python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06c_bnbs_stats.log 2>&1 || exit 18
