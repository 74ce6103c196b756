# Config C5 (BASELINE configs[4]: 5k-arc network, 512 scenarios): DD parity vs the oracle,
# per-phase diagnostics of one 1024-record launch, and a bench line with the subproblem leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "bench_workload" --timeout 200 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/relax_diag.py --config C5 --nodes ${C5N:-1024} > gpurun_out/c5_diag.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config C5 --nodes ${C5N:-1024} --steps 5 --warmup 1 --no-cpu --sub-paths 8 > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
