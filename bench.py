#!/usr/bin/env python3
"""B&B-node relaxations/s on the 1k-arc, 256-scenario synthetic instance (BASELINE.json).

One step = NodeExplorer::process (NodeExplorer.cpp:915-986) for a whole batch of open
nodes, on the device: build every relaxed DD, sweep the 16 feasibility + 64 optimality
cuts of the pool over it (newest first), apply the reference's edits, and write the
cutset children as frontier records (k_relax + k_scan2 + k_emit_children).  Inputs
(network tables, cut rows, the open-node records) are resident in HBM before the
timed region.  Exact DDs stop at the scenario-subproblem hand-off (status
NEEDS_SUBPROBLEM, argmax path written) -- see DESIGN.md.

Workload (config C4): seeded layered instance with 1000 arcs and 256
scenarios, 16F + 64O synthetic cuts (tests2.cpp:259-286 recipe), a BFS frontier of
open nodes from the root, incumbent = 40th percentile of the frontier's bounds.
With N ranks every rank relaxes its own slice of a frontier N times as large
(weak scaling, no collective on the data path; the per-step time is the max over
ranks).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run and this script reads RANK / LOCAL_RANK / WORLD_SIZE.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "B&B-node relaxations/sec + achieved HBM GB/s, 1k-arc 256-scenario synthetic"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=8192, help="open nodes per GPU per step")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--n-feas", type=int, default=16)
    ap.add_argument("--n-opt", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-sample", type=int, default=2048)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-tag", default="r02")
    ap.add_argument("--sub-paths", type=int, default=32, help="subproblem leg: random full-matching paths (0: skip)")
    ap.add_argument("--cpu-sub-seconds", type=float, default=8.0)
    ap.add_argument("--c5-nodes", type=int, default=1024,
                    help="config-5 leg (5k arcs, 512 scenarios): open nodes relaxed per step (0: skip)")
    ap.add_argument("--c5-paths", type=int, default=4, help="config-5 leg: subproblem paths x 512 scenarios")
    ap.add_argument("--mode", choices=["relax", "bnb"], default="relax",
                    help="relax: the headline batch relaxation; bnb: the device B&B (config C3) for --bnb-seconds")
    ap.add_argument("--bnb-config", default="C3")
    ap.add_argument("--bnb-seconds", type=float, default=30.0)
    ap.add_argument("--bnb-lb", choices=["zero", "gen"], default="zero",
                    help="zero: drop the generator's sink lower bounds so the instance is feasible and "
                         "incumbents / optimality cuts appear (with them most C3 paths are infeasible)")
    return ap.parse_args()


def lib_sha256() -> str:
    import hashlib
    path = os.path.join(ROOT, "sgufp_solver_amd", "lib", "libsgufp_hip.so")
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


# FETCH_SIZE correction on gfx950, measured by tools/calib (profiles/r02_fetch_calibration.json):
# a coalesced 1 GiB stream of 4-, 8- or 16-byte loads per lane reports exactly 0.5 GiB of
# FETCH_SIZE, and WRITE_SIZE reports stores of every width at 1.00 (1-byte stores 1.01).
FETCH_CORRECTION = 2.0


def workload_key(args) -> str:
    """The bench workload a PMC profile belongs to (profiles/<tag>_pmc_*/workload.txt)."""
    return f"{args.config}:seed{args.seed}:nodes{args.nodes}:pool{args.n_feas}F+{args.n_opt}O"


def pmc_traffic(tag: str, workload: str, kernel: str = "k_relax"):
    """(HBM bytes per launch of `kernel`, source) from the rocprofv3 --pmc CSVs of the same
    bench command (profiles/<tag>_pmc_fetch/*counter_collection.csv, profiles/<tag>_pmc_write/...),
    only when they were collected with this very library (lib.sha256 next to the CSVs) on
    this very workload (workload.txt); otherwise (None, reason).  FETCH_SIZE x FETCH_CORRECTION + WRITE_SIZE; both count the
    L2's fabric-side requests (Infinity-Cache hits included), so this is L2-miss traffic."""
    want = lib_sha256()
    for sub in ("pmc_fetch", "pmc_write"):
        shafile = os.path.join(ROOT, "profiles", f"{tag}_{sub}", "lib.sha256")
        if not os.path.exists(shafile):
            return None, f"profiles/{tag}_{sub}/lib.sha256 missing"
        with open(shafile) as fh:
            if fh.read().strip() != want:
                return None, f"profiles/{tag}_{sub} was collected with another build of libsgufp_hip.so"
        wfile = os.path.join(ROOT, "profiles", f"{tag}_{sub}", "workload.txt")
        if not os.path.exists(wfile):
            return None, f"profiles/{tag}_{sub}/workload.txt missing"
        with open(wfile) as fh:
            if fh.read().strip() != workload:
                return None, f"profiles/{tag}_{sub} was collected on another workload"
    def load(pattern, counter):
        # only the bench launches (largest grid): the 1024-node probe launch is excluded
        rows = []
        for path in glob.glob(os.path.join(ROOT, "profiles", pattern)):
            import csv
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        rows.append((int(row["Grid_Size"]), float(row["Counter_Value"])))
        if not rows:
            return []
        g = max(r[0] for r in rows)
        return [v for gs, v in rows if gs == g]
    f = load(f"{tag}_pmc_fetch/*counter_collection.csv", "FETCH_SIZE")
    w = load(f"{tag}_pmc_write/*counter_collection.csv", "WRITE_SIZE")
    if not f or not w:
        return None, f"no {kernel} rows in profiles/{tag}_pmc_*"
    src = (f"profiles/{tag}_pmc_fetch + {tag}_pmc_write (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of "
           f"bench.py --steps 2, libsgufp_hip.so sha256 {want[:16]}); FETCH_SIZE x {FETCH_CORRECTION}")
    return (FETCH_CORRECTION * np.mean(f) + np.mean(w)) * 1024.0, src


def bnb_main(args):
    """Full B&B on the device (BASELINE configs[2]: 1k-arc network, 64 scenarios): the
    DDSolver from the root record Node{} with no incumbent, for --bnb-seconds after a short
    warm-up run; relaxations/s = NodeExplorer::process calls (exact-leaf refinement loops
    with the device subproblem included) per second of the timed run.  With N ranks the
    search is shared (incumbent all-reduce, cut all-gather, work stealing; strong scaling)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MIN
    from sgufp_solver_amd.solver import DDSolver
    cfg = instance.CONFIGS[args.bnb_config]
    inst = instance.generate(cfg, args.seed)
    if args.bnb_lb == "zero":
        inst.lb[:] = 0
    work = tempfile.mkdtemp(prefix=f"sgufp_bnb_r{rank}_")
    net = os.path.join(work, "net.txt")
    inst.write(net)
    # a round (and its refinement loops) can run for minutes: keep a heartbeat on stderr
    import threading
    t_hb = time.perf_counter()

    def heartbeat():
        while True:
            time.sleep(20.0)
            print(f"bnb: running, {time.perf_counter() - t_hb:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    solver = DDSolver(net, device=local, max_batch=args.nodes, verbose=False, time_budget=2.0, progress=10.0)
    solver.start_solver(DOUBLE_MIN)                        # warm-up (kernels, allocations)
    solver.eng.clear_cuts()
    solver.eng.set_timing(True)
    solver.time_budget = args.bnb_seconds
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    z = solver.start_solver(DOUBLE_MIN)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    c = dict(solver.counters)
    if dist:
        t = torch.tensor([elapsed] + [float(c[k]) for k in sorted(c)], dtype=torch.float64,
                         device="cuda" if torch.cuda.is_available() else "cpu")
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        c = {k: int(v) for k, v in zip(sorted(c), t[1:].tolist())}
    line = {
        "metric": "device B&B: node relaxations/s (NodeExplorer::process incl. exact-leaf subproblems)",
        "value": round(c["relaxed"] / elapsed, 2), "unit": "relaxations/s", "n_gpus": world,
        "seconds": round(elapsed, 3), "rounds": solver.rounds, "complete": solver.complete, "incumbent": z,
        "higher_is_better": True, "scaling": "strong", "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{args.bnb_config}: {cfg.n_arcs}-arc layered network, {inst.scenarios} scenarios"
                               f"{' (lower bounds 0)' if args.bnb_lb == 'zero' else ''}, root record, no incumbent, "
                               f"up to {args.nodes} records per round",
                   "instance_seed": args.seed, "total_layers": int(solver.eng.info.total_layers)},
        "counters": c,
        "pool": [solver.eng.cuts_count(1), solver.eng.cuts_count(0)],
        "subproblems_per_s": round(c["subproblems"] / elapsed, 2),
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    solver.eng.close()
    if dist:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.mode == "bnb":
        return bnb_main(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
    import torch

    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import frontier, instance, pools

    cfg = instance.CONFIGS[args.config]
    inst = instance.generate(cfg, args.seed)
    work = tempfile.mkdtemp(prefix=f"sgufp_bench_r{rank}_")
    net = os.path.join(work, "net.txt")
    inst.write(net)
    pool = pools.synthetic_pool(inst, args.n_feas, args.n_opt, args.seed)

    n = args.nodes
    eng = E.Engine(net, local, max(n, 1024))
    if rank == 0:
        print(f"[bench] L={eng.info.total_layers} slots={eng.info.max_batch} node_cap={eng.info.node_capacity} "
              f"arc_cap={eng.info.arc_capacity} scratch={eng.info.scratch_bytes / 2**30:.2f} GiB", file=sys.stderr)
    full = frontier.bfs_frontier(eng, n * world)          # identical on every rank
    eng.add_cuts(pool)
    # incumbent: 40th percentile of the (finite) bounds of the first 1024 records
    probe = E.batch_slice(full, np.arange(min(1024, full.n)))
    eng.upload(probe)
    eng.relax_async(pools.DOUBLE_MIN)
    eng.sync()
    st, ex, lb, ub, nc = eng.results_arrays()
    fin = ub[(st == 0) | (st == 3)]
    incumbent = float(np.percentile(fin, 40)) if fin.size else 0.0
    mine = E.batch_slice(full, np.arange(rank * n, min(full.n, (rank + 1) * n)))
    eng.upload(mine)

    eng.set_timing(True)
    for _ in range(args.warmup):
        eng.relax_async(incumbent)
        eng.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    relax_ms = []
    emit_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.relax_async(incumbent)
        eng.sync()
        a, b = eng.last_timing()
        relax_ms.append(a)
        emit_ms.append(b)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-launch algorithmic bytes: 6A + sum_cuts(14A + 8N) + record in
    st, ex, lb, ub, nc = eng.results_arrays()
    dn, da, dl, sw = eng.stats()
    g = mine.gl.astype(np.float64)
    ns = np.diff(mine.states_off).astype(np.float64)
    r_in = 2 * g + 2 * ns + 24
    bytes_relax = float(np.sum(6.0 * da + sw * (14.0 * da + 8.0 * dn) + r_in))
    ch = eng.children_batch()
    r_out = float(np.sum(2 * ch.gl.astype(np.float64) + 2 * np.diff(ch.states_off) + 24)) if ch.n else 0.0
    t_relax = float(np.mean(relax_ms)) / 1e3
    achieved = bytes_relax / t_relax / 1e9
    traffic, traffic_src = pmc_traffic(args.profile_tag, workload_key(args))

    total_nodes = mine.n * world
    value = total_nodes * args.steps / elapsed
    sub = subproblem_leg(eng, inst, net, args) if rank == 0 else None
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "relaxations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: {cfg.n_arcs}-arc layered network, {inst.scenarios} scenarios, "
                        f"{args.n_feas}F+{args.n_opt}O pool, BFS frontier of {n} open nodes per GPU",
            "instance_seed": args.seed, "nodes_per_gpu": n, "incumbent": incumbent,
            "total_layers": int(eng.info.total_layers),
            "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
            "avg_dd_nodes": float(np.mean(dn)), "avg_dd_arcs": float(np.mean(da)),
            "avg_sweeps": float(np.mean(sw)), "children_per_step": int(ch.n),
            "parallelism": f"frontier shards x{world}",
        },
        "hbm_gbps_algorithmic": round(achieved, 2),
        "roofline": {
            # the roofline that bounds this class of kernel (no MFMA work); the kernel itself
            # is limited by instruction issue and LDS latency, not by HBM
            "bound": "hbm",
            "limiter": "latency/issue (measured HBM traffic is a fraction of the algorithmic bytes)",
            # SURVEY 8(d)'s byte model streams every (arc, cut) operand from HBM; the kernel
            # serves most of them from LDS / L2 (topology staged once per cut batch), so the
            # model's rate can pass the HBM peak -- frac_traffic is the measured utilisation
            "byte_model": "SURVEY 8(d): 6A + sum over applied cuts (14A + 8N) + records; not HBM traffic",
            "kernel": "k_relax",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_gbps": round(traffic / t_relax / 1e9, 2) if traffic else None,
            "frac_traffic": round(traffic / t_relax / 1e9 / HBM_PEAK_GBPS, 4) if traffic else None,
            "traffic_source": traffic_src,
            "bytes_per_launch": bytes_relax,
            "avg_launch_ms": round(t_relax * 1e3, 4),
            "emit_ms": round(float(np.mean(emit_ms)), 4),
            "children_record_bytes": r_out,
        },
        "cpu_baseline": None,
        "subproblem": sub,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(work, net, pool, mine, incumbent, args)
        if sub is not None:
            i0, n0 = sub["_inst0"]
            sub["cpu_baseline"] = cpu_subproblem_baseline(inst, net, sub["_paths"], args, i0, n0)
    if sub is not None:
        sub.pop("_paths", None)
        sub.pop("_inst0", None)
    eng.close()
    if rank == 0 and world == 1 and args.config == "C4" and args.c5_nodes > 0:
        line["config5"] = config5_leg(args, work)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def config5_leg(args, work):
    """BASELINE configs[4]: the 5k-arc, 512-scenario instance with cut generation in the loop.
    Relaxation rate of a BFS frontier of --c5-nodes records under a 16F + 64O pool (same
    timing as the headline, k_relax on the library's stream), and the scenario subproblem
    (k_sub_scenario + k_sub_reduce) on --c5-paths random full matchings x 512 scenarios with
    lower bounds 0 (every scenario optimal: full max-reward flows, optimality cuts)."""
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import frontier, instance, pools
    cfg = instance.CONFIGS["C5"]
    inst = instance.generate(cfg, args.seed)
    inst.lb[:] = 0
    net = os.path.join(work, "net_c5.txt")
    inst.write(net)
    pool = pools.synthetic_pool(inst, args.n_feas, args.n_opt, args.seed)
    n = args.c5_nodes
    eng = E.Engine(net, 0, n)
    fr = frontier.bfs_frontier(eng, n)
    eng.add_cuts(pool)
    eng.upload(fr)
    eng.relax_async(pools.DOUBLE_MIN)
    eng.sync()
    st, ex, lb, ub, nc = eng.results_arrays()
    fin = ub[(st == 0) | (st == 3)]
    inc = float(np.percentile(fin, 40)) if fin.size else 0.0
    eng.set_timing(True)
    eng.relax_async(inc)
    eng.sync()
    steps = 5
    ms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.relax_async(inc)
        eng.sync()
        ms.append(eng.last_timing()[0])
    wall = time.perf_counter() - t0
    st, ex, lb, ub, nc = eng.results_arrays()
    dn, da, dl, sw = eng.stats()
    out = {"workload": f"C5: {cfg.n_arcs}-arc layered network, {inst.scenarios} scenarios, {args.n_feas}F+{args.n_opt}O "
                       f"pool, BFS frontier of {fr.n} open nodes", "instance_seed": args.seed, "incumbent": inc,
           "relaxations_per_s": round(fr.n * steps / wall, 2), "k_relax_ms": round(float(np.mean(ms)), 4),
           "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
           "avg_dd_nodes": float(np.mean(dn)), "avg_sweeps": float(np.mean(sw))}
    if args.c5_paths > 0:
        _, la, _ = E.probe_network(net)
        rng = np.random.default_rng(args.seed + 7)
        paths = [instance.random_matching_path(inst, la, rng) for _ in range(args.c5_paths)]
        eng.subproblem(paths)                                  # warm-up
        t0 = time.perf_counter()
        typ, _, _, _ = eng.subproblem(paths)
        t = time.perf_counter() - t0
        out["subproblem"] = {"kernel": "k_sub_scenario", "paths": len(paths), "scenarios": int(inst.scenarios),
                             "lower_bounds": 0, "ms_per_call": round(t * 1e3, 2),
                             "scenario_lps_per_s": round(len(paths) * inst.scenarios / t, 1),
                             "cut_types": {str(k): int(v) for k, v in zip(*np.unique(typ, return_counts=True))}}
    eng.close()
    return out


def subproblem_leg(eng, inst, net, args):
    """The exact-leaf half of a relaxation: GuroSolver::solveSubProblem (grb.cpp:139-360)
    on the device (k_sub_scenario + k_sub_reduce) for --sub-paths random full matchings,
    every scenario; scenario LPs per second of the synchronous call (paths uploaded, cut
    rows downloaded).  Two cases: the bench instance itself (its sink-arc lower bounds
    make most matchings infeasible: Farkas rays, feasibility cuts) and the same network
    with lower bounds 0 (every scenario optimal: full max-reward flows, optimality cuts)."""
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import instance
    if args.sub_paths <= 0:
        return None
    _, la, _ = E.probe_network(net)
    rng = np.random.default_rng(args.seed + 7)
    paths = [instance.random_matching_path(inst, la, rng) for _ in range(args.sub_paths)]
    inst0 = instance.generate(instance.CONFIGS[args.config], args.seed)
    inst0.lb[:] = 0
    net0 = os.path.join(os.path.dirname(net), "net_lb0.txt")
    inst0.write(net0)
    out = {"kernel": "k_sub_scenario", "paths": len(paths), "scenarios": int(inst.scenarios), "_paths": paths}
    eng0 = E.Engine(net0, eng.device, 64)
    for name, e in (("generated_bounds", eng), ("lower_bounds_0", eng0)):
        e.subproblem(paths)                                 # warm-up
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            typ, _, _, _ = e.subproblem(paths)
            ts.append(time.perf_counter() - t0)
        t = float(np.mean(ts))
        lps = len(paths) * inst.scenarios
        out[name] = {"ms_per_call": round(t * 1e3, 3), "scenario_lps_per_s": round(lps / t, 1),
                     "paths_per_s": round(len(paths) / t, 2),
                     "cut_types": {str(k): int(v) for k, v in zip(*np.unique(typ, return_counts=True))}}
    eng0.close()
    out["_inst0"] = (inst0, net0)
    return out


def cpu_subproblem_baseline(inst, net, paths, args, inst0=None, net0=None):
    """The reference solves each scenario LP with Gurobi 11 (absent here): its dual LP
    restated (oracle/subproblem_oracle.py) and solved with scipy HiGHS on one core, on a
    bounded sample of the same (path, scenario) pairs (lower bounds 0 case when given)."""
    from oracle import subproblem_oracle as so
    from sgufp_solver_amd import engine as E
    if inst0 is not None:
        inst, net = inst0, net0
    _, la, _ = E.probe_network(net)
    sn = so.from_instance(inst, la)
    done, t0 = 0, time.perf_counter()
    for p in paths:
        y = so.ybar_of_path(sn, p)
        for s in range(inst.scenarios):
            so.dual_lp(sn, y, s)
            done += 1
            if time.perf_counter() - t0 > args.cpu_sub_seconds:
                break
        if time.perf_counter() - t0 > args.cpu_sub_seconds:
            break
    t = time.perf_counter() - t0
    return {"value": round(done / t, 2), "unit": "scenario LPs/s", "cores": 1, "kind": "port",
            "sample": f"{done} (path, scenario) dual LPs of the reference formulation"
                      f"{' (lower bounds 0)' if inst0 is not None else ''}, scipy HiGHS, {t:.1f} s"}


def cpu_baseline(work, net, pool, batch, incumbent, args):
    """The reference's own RelaxedDDNew (oracle/_ref/ref_dd, built from its sources)
    when present, else the clean-room port, on the host cores, bounded sample."""
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import pools
    sample = E.batch_slice(batch, np.arange(min(args.cpu_sample, batch.n)))
    nodes = os.path.join(work, "nodes.txt")
    cuts = os.path.join(work, "cuts.txt")
    pools.write_nodes(nodes, E.batch_to_records(sample))
    pools.write_pool(cuts, pool)
    threads = max(1, min(16, os.cpu_count() or 1))
    for kind, exe in (("reference", os.path.join(ROOT, "oracle", "_ref", "ref_dd")),
                      ("port", os.path.join(ROOT, "oracle", "_build", "dd_oracle"))):
        if not os.path.exists(exe):
            continue
        r = subprocess.run([exe, "time", net, cuts, nodes, incumbent.hex(), str(threads), str(args.cpu_seconds)],
                           capture_output=True, text=True, timeout=args.cpu_seconds * 4 + 120)
        if r.returncode != 0:
            continue
        out = json.loads(r.stdout.strip().splitlines()[-1])
        cpu_model = ""
        try:
            with open("/proc/cpuinfo") as fh:
                cpu_model = next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
        except Exception:
            pass
        return {"value": round(out["relaxations"] / out["seconds"], 2), "unit": "relaxations/s", "cores": threads,
                "kind": kind, "cpu": cpu_model,
                "sample": f"{out['relaxations']} of the first {sample.n} open nodes of the same frontier, same pool and "
                          f"incumbent, {out['seconds']:.1f} s on {threads} threads"}
    return None


if __name__ == "__main__":
    main()
