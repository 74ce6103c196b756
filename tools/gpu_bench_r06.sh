#!/bin/bash
# round-6 end: headline kernel stats, HBM (FETCH / WRITE) and issue (SQ) counter passes of the
# bench command; the seeded B&B leg's kernel shares and its dominant kernels' issue / LDS
# counters (bnb_seeded roofline block).  The bench line (tools/gpu_bench_r05_line.sh) reads them
# back from profiles/ when the library matches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06
ONLY="--no-cpu --no-parity --sub-paths 0 --c5-nodes 0 --bnb-seeded-width 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-parity-rounds 0 --bnb-gen-seconds 0 --cpp-leg-seconds 0 --bnb-parity-survivor-pool 0"
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
mkdir -p gpurun_out
stamp() {
  sha256sum sgufp_solver_amd/lib/libsgufp_hip.so | cut -d' ' -f1 > gpurun_out/${TAG}_$1/lib.sha256
  python3 tools/kernel_src_sha256.py > gpurun_out/${TAG}_$1/src.sha256
  echo "$2" > gpurun_out/${TAG}_$1/workload.txt
}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o run -- python3 bench.py --steps 5 --warmup 2 $ONLY > gpurun_out/${TAG}_stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 $ONLY > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 $ONLY > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d gpurun_out/${TAG}_pmc_issue -o run -- python3 bench.py --steps 2 --warmup 1 $ONLY > gpurun_out/${TAG}_pmc_issue.log 2>&1 || exit $?
for d in pmc_fetch pmc_write pmc_issue; do stamp $d "C4:seed1:nodes8192:pool16F+64O"; done
# (SGUFP_EXACT_STATS: the leaf passes' byte-model counters, [exact-cum] on stderr, kept beside each profile)
SGUFP_EXACT_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bnbs_stats -o run -- python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/${TAG}_bnbs_stats.log 2>&1 || exit $?
grep "exact-cum" gpurun_out/${TAG}_bnbs_stats.log | tail -n 3 > gpurun_out/${TAG}_bnbs_stats/exact_cum.log
SGUFP_EXACT_STATS=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_bnbs_pmc_fetch -o run -- python3 bench.py $BNBS --bnb-seconds 12 > gpurun_out/${TAG}_bnbs_pmc_fetch.log 2>&1 || exit $?
grep "exact-cum" gpurun_out/${TAG}_bnbs_pmc_fetch.log | tail -n 3 > gpurun_out/${TAG}_bnbs_pmc_fetch/exact_cum.log
SGUFP_EXACT_STATS=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_bnbs_pmc_write -o run -- python3 bench.py $BNBS --bnb-seconds 12 > gpurun_out/${TAG}_bnbs_pmc_write.log 2>&1 || exit $?
grep "exact-cum" gpurun_out/${TAG}_bnbs_pmc_write.log | tail -n 3 > gpurun_out/${TAG}_bnbs_pmc_write/exact_cum.log
python3 tools/compact_pmc.py gpurun_out/${TAG}_bnbs_pmc_fetch/*counter_collection.csv gpurun_out/${TAG}_bnbs_pmc_write/*counter_collection.csv
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    --output-format csv -d gpurun_out/${TAG}_bnbs_pmc_issue -o run -- python3 bench.py $BNBS --bnb-seconds 8 > gpurun_out/${TAG}_bnbs_pmc_issue.log 2>&1 || exit $?
for d in bnbs_stats bnbs_pmc_issue bnbs_pmc_fetch bnbs_pmc_write; do stamp $d "bnb:C4:seed1:zero:heuristic128:batch1024"; done
python3 tools/compact_pmc.py gpurun_out/${TAG}_bnbs_pmc_issue/*counter_collection.csv
# the subproblem alone (C4 32 paths x 256 scenarios, cold): issue / LDS counters of k_sub_scenario
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    --output-format csv -d gpurun_out/${TAG}_sub_pmc -o run -- python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/${TAG}_sub_pmc.log 2>&1 || exit $?
stamp sub_pmc "sub:C4:seed1:paths32:scenarios256:cold"
python3 tools/compact_pmc.py gpurun_out/${TAG}_sub_pmc/*counter_collection.csv
rm -f gpurun_out/${TAG}_*/run_kernel_trace.csv   # (per-dispatch rows: kept out of profiles/)
# the bench line reads profiles/: copy the fresh counters there on the box as well
for d in stats pmc_fetch pmc_write pmc_issue bnbs_stats bnbs_pmc_issue bnbs_pmc_fetch bnbs_pmc_write sub_pmc; do rm -rf profiles/${TAG}_$d; cp -r gpurun_out/${TAG}_$d profiles/; done
ls gpurun_out/${TAG}_bnbs_stats
