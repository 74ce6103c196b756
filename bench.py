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
With N ranks every rank relaxes its own slice of a frontier N times as large (weak
scaling) and every step ends with the B&B round's exchanges over RCCL: the incumbent
all-reduce(MAX) and the all-gather of the round's new cut rows (shards.py); the
per-step time is the max over ranks.

Beside the headline the line carries: `parity` (the timed step's results for the first
--cpu-sample records against the reference's own RelaxedDDNew on the same records, bit for
bit), `cpu_baseline` (that reference run's rate on the host cores), `roofline` (PMC-counted
HBM bytes of this build per k_relax launch, with the issue counters of the same build),
`subproblem` (the scenario LP kernels alone), `bnb` / `bnb_seeded` (the device B&B with its
exact-leaf subproblems on the same 256-scenario network, without an incumbent / seeded by the
restricted-DD heuristic inside the timed region), `bnb_parity` (rounds of the seeded search
checked against the reference under the search's own Benders pools, oracle/bnb_parity.py) and
`config5` (BASELINE configs[4]: 5k arcs, 512 scenarios, relaxation with a 256-record parity
block, subproblem, B&B with cut generation).  With N > 1 ranks `bnb_multi` is the seeded C4
search strong-scaled over the N frontier shards (incumbent all-reduce, cut-row all-gather and
work sharing every round; through the library's own RCCL communicator, shard.cpp, when the
backend is nccl).  Progress goes to stderr; stdout carries the one JSON line.

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
    ap.add_argument("--profile-tag", default="r06")
    ap.add_argument("--sub-paths", type=int, default=32, help="subproblem leg: random full-matching paths (0: skip)")
    ap.add_argument("--cpu-sub-seconds", type=float, default=8.0)
    ap.add_argument("--c5-nodes", type=int, default=4096,
                    help="config-5 leg (5k arcs, 512 scenarios): open nodes relaxed per step (0: skip)")
    ap.add_argument("--c5-paths", type=int, default=4, help="config-5 leg: subproblem paths x 512 scenarios")
    ap.add_argument("--c5-parity", type=int, default=256,
                    help="config-5 leg: records of the timed step checked against the reference (0: none)")
    ap.add_argument("--mode", choices=["relax", "bnb"], default="relax",
                    help="relax: the headline batch relaxation; bnb: the device B&B (config C3) for --bnb-seconds")
    ap.add_argument("--bnb-config", default="C3")
    ap.add_argument("--bnb-seconds", type=float, default=30.0)
    ap.add_argument("--bnb-lb", choices=["zero", "gen"], default="zero",
                    help="zero: drop the generator's sink lower bounds so the instance is feasible and "
                         "incumbents / optimality cuts appear (with them most C3 paths are infeasible)")
    ap.add_argument("--round-seconds", type=float, default=5.0,
                    help="B&B: a round's exact-leaf refinement loops are deferred after this many seconds")
    ap.add_argument("--bnb-streams", type=int, default=1,
                    help="--mode bnb: frontier shards on the device (one context / stream / host thread each)")
    ap.add_argument("--bnb-heuristic", type=int, default=0,
                    help="--mode bnb: seed the incumbent with the restricted-DD heuristic of this width (0: none)")
    ap.add_argument("--bnb-seeded-width", type=int, default=128,
                    help="B&B leg with the incumbent seeded by the restricted-DD heuristic of this width (0: skip)")
    ap.add_argument("--bnb-leg-seconds", type=float, default=20.0,
                    help="headline line: seconds of the C4 / 256-scenario B&B leg (0: skip)")
    ap.add_argument("--bnb-gen-seconds", type=float, default=20.0,
                    help="headline line: seconds of the seeded C4 B&B with the generator's lower bounds kept "
                         "(bnb_gen: infeasible scenarios, feasibility cuts in the loop; 0: skip)")
    ap.add_argument("--cpp-leg-seconds", type=float, default=20.0,
                    help="headline line: seconds of the seeded C4 B&B through the C++ host API (Inavap::DDSolver, "
                         "tests/host/host_api_test search; 0: skip)")
    ap.add_argument("--bnb-parity-survivor-pool", type=int, default=20000,
                    help="bnb_parity leg: optimality cuts the unseeded search accumulates before its non-exact "
                         "survivors are checked (0: skip)")
    ap.add_argument("--c5-bnb-seconds", type=float, default=30.0,
                    help="config-5 leg: seconds of the C5 / 512-scenario B&B with cut generation (0: skip)")
    ap.add_argument("--no-parity", action="store_true", help="skip the reference parity check of the timed batch")
    ap.add_argument("--bnb-parity-pool", type=int, default=10000,
                    help="bnb_parity leg: optimality cuts the seeded search accumulates before the check")
    ap.add_argument("--bnb-parity-rounds", type=int, default=3,
                    help="0: skip the bnb_parity leg (the seeded device B&B checked against the reference under its "
                         "own cuts, at --bnb-parity-pool optimality cuts)")
    return ap.parse_args()


def lib_sha256() -> str:
    import hashlib
    path = os.path.join(ROOT, "sgufp_solver_amd", "lib", "libsgufp_hip.so")
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


# the sources of k_relax (its HBM traffic depends on them, not on the bits of one build)
KERNEL_SOURCES = ("dd_kernels.hip", "dd_device.hpp", "wave.hpp")


def kernel_src_sha256() -> str:
    """sha256 over k_relax's sources and the hipcc flags (tools/kernel_src_sha256.py writes the
    same value next to the PMC CSVs)."""
    import hashlib
    sys.path.insert(0, ROOT)
    from sgufp_solver_amd.build import COMMON
    h = hashlib.sha256(" ".join(f for f in COMMON if not f.startswith("-I")).encode())
    for name in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "sgufp_solver_amd", "csrc", name), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def profile_matches(d: str):
    """'library' / 'sources' when the PMC profile directory d was collected with this very
    libsgufp_hip.so / with k_relax built from these very sources, else None."""
    for fname, want, what in (("lib.sha256", lib_sha256, "library"), ("src.sha256", kernel_src_sha256, "sources")):
        path = os.path.join(d, fname)
        if os.path.exists(path):
            with open(path) as fh:
                if fh.read().strip() == want():
                    return what
    return None


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
    match = None
    for sub in ("pmc_fetch", "pmc_write"):
        match = profile_matches(os.path.join(ROOT, "profiles", f"{tag}_{sub}"))
        if match is None:
            return None, f"profiles/{tag}_{sub} was collected with another k_relax (library and source hashes differ)"
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
    ident = (f"libsgufp_hip.so sha256 {lib_sha256()[:16]}" if match == "library"
             else f"k_relax sources sha256 {kernel_src_sha256()[:16]}")
    src = (f"profiles/{tag}_pmc_fetch + {tag}_pmc_write (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of "
           f"bench.py --steps 2, {ident}); FETCH_SIZE x {FETCH_CORRECTION}")
    return (FETCH_CORRECTION * np.mean(f) + np.mean(w)) * 1024.0, src


def pmc_issue(tag: str, workload: str, kernel: str = "k_relax"):
    """Issue-side counters of `kernel` (profiles/<tag>_pmc_issue, same build and workload as
    the HBM passes): per launch the wave-instructions issued and where the waves' cycles went.
    SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY count quad-cycles and partition the
    waves' lifetime (MI355X_MICROARCH.md, rocprofv3 PMC slots)."""
    d = os.path.join(ROOT, "profiles", f"{tag}_pmc_issue")
    try:
        if profile_matches(d) is None or open(os.path.join(d, "workload.txt")).read().strip() != workload:
            return None
    except OSError:
        return None
    import csv
    rows = []
    for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(path) as fh:
            rows += [r for r in csv.DictReader(fh) if kernel in r.get("Kernel_Name", "")]
    if not rows:
        return None
    g = max(int(r["Grid_Size"]) for r in rows)
    acc = {}
    for r in rows:
        if int(r["Grid_Size"]) == g:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    c = {k: float(np.mean(v)) for k, v in acc.items()}
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if not wc:
        return None
    waves = c.get("SQ_WAVES", 1.0)
    return {"source": f"profiles/{tag}_pmc_issue (rocprofv3 --pmc SQ_*)",
            "valu_insts_per_launch": c.get("SQ_INSTS_VALU"), "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
            "valu_insts_per_wave": round(c.get("SQ_INSTS_VALU", 0.0) / waves),
            "active_frac": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
            "wait_frac": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 4),
            "issue_stall_frac": round(c.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4),
            "cycles_per_wave_instruction": round(4.0 * wc / max(1.0, c.get("SQ_INSTS_VALU", 0.0) +
                                                                 c.get("SQ_INSTS_SALU", 0.0)), 2)}


def bnb_profile_block(tag: str):
    """The north-star loop's own profile: for the seeded B&B leg's command
    (bench.py --mode bnb, C4 / 256, seeded by the width-128 heuristic), from
    profiles/<tag>_bnbs_stats (rocprofv3 --kernel-trace --stats: every kernel's share of the GPU
    time) and profiles/<tag>_bnbs_pmc_issue (rocprofv3 --pmc SQ_*: issue, wait and LDS counters
    summed over every dispatch of the dominant kernels), only when they were collected with this
    very library (lib.sha256 next to them); else None."""
    import csv
    d = os.path.join(ROOT, "profiles", f"{tag}_bnbs_stats")
    dp = os.path.join(ROOT, "profiles", f"{tag}_bnbs_pmc_issue")
    if profile_matches(d) != "library":
        return None
    shares = {}
    for path in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                name = r["Name"].split("(")[0].replace("void ", "").strip()
                shares[name] = shares.get(name, 0.0) + float(r["TotalDurationNs"])
    if not shares:
        return None
    tot = sum(shares.values())
    top = sorted(shares.items(), key=lambda kv: -kv[1])
    out = {"source": f"profiles/{tag}_bnbs_stats (rocprofv3 --kernel-trace --stats of bench.py --mode bnb "
                     f"--bnb-config C4 --bnb-heuristic 128, libsgufp_hip.so sha256 {lib_sha256()[:16]})",
           "gpu_seconds": round(tot * 1e-9, 3),
           "kernel_shares": {k: round(v / tot, 4) for k, v in top[:6]},
           "dominant_kernel": top[0][0], "dominant_share": round(top[0][1] / tot, 4)}
    if profile_matches(dp) == "library":
        acc = {}
        for path in glob.glob(os.path.join(dp, "*counter_collection.csv")):
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                    acc.setdefault(name, {}).setdefault(r["Counter_Name"], 0.0)
                    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        per = {}
        for k, _ in top[:3]:
            c = acc.get(k)
            if not c or not c.get("SQ_WAVE_CYCLES"):
                continue
            wc = c["SQ_WAVE_CYCLES"]
            insts = c.get("SQ_INSTS_VALU", 0.0) + c.get("SQ_INSTS_SALU", 0.0)
            per[k] = {"active_frac": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
                      "wait_frac": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 4),
                      "lds_active_frac": round(c.get("SQ_ACTIVE_INST_LDS", 0.0) / wc, 4),
                      "lds_bank_conflict_frac": round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                                                      max(1.0, c.get("SQ_ACTIVE_INST_LDS", 0.0)), 4),
                      "valu_insts": c.get("SQ_INSTS_VALU"), "salu_insts": c.get("SQ_INSTS_SALU"),
                      "lds_insts": c.get("SQ_INSTS_LDS"),
                      "cycles_per_wave_instruction": round(4.0 * wc / max(1.0, insts), 2)}
        out["issue"] = per
        out["issue_source"] = (f"profiles/{tag}_bnbs_pmc_issue (rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY "
                               f"SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS "
                               f"SQ_LDS_BANK_CONFLICT, same command and library; wave cycles in quad-cycles)")
    leaf = leaf_roofline(tag, top[0][0], shares.get(top[0][0], 0.0), d)
    if leaf:
        out["dominant_roofline"] = leaf
    out["bound"] = "issue/latency (waves parked on dependent LDS / memory round trips; see issue)"
    return out


def _exact_cum(path):
    """The last [exact-cum] line of a log (SGUFP_EXACT_STATS=1): (pass-blocks, row-blocks, bytes)."""
    last = None
    if os.path.exists(path):
        with open(path, errors="replace") as fh:
            for ln in fh:
                if ln.startswith("[exact-cum]"):
                    last = ln.split()
    if not last:
        return None
    return int(last[3]), int(last[5]), float(last[7])


def leaf_roofline(tag: str, kernel: str, kernel_ns: float, stats_dir: str):
    """Roofline of the seeded leg's dominant kernel when it is the exact leaf passes
    (k_exact_leaf): algorithmic bytes = per swept 64-cut block of a pass its staged coefficient
    rows plus the root-fold column, 64 x 8 B each (the kernel's own counters, summed over the leg:
    SGUFP_EXACT_STATS [exact-cum] in the stats run's log), over the kernel's total time in the same
    run; HBM traffic per pass-block from the FETCH_SIZE / WRITE_SIZE passes of the same command
    (profiles/<tag>_bnbs_pmc_fetch / _write, each with its own [exact-cum] counts)."""
    import csv
    if "k_exact_leaf" not in kernel or kernel_ns <= 0:
        return None
    cum = _exact_cum(os.path.join(stats_dir, "exact_cum.log"))
    if not cum:
        return None
    blocks, rows, model = cum
    out = {"kernel": kernel, "model": "per pass-block: (staged rows + 1 root-fold column) x 64 cuts x 8 B",
           "pass_blocks": blocks, "row_blocks": rows, "model_bytes": model,
           "kernel_seconds": round(kernel_ns * 1e-9, 4),
           "achieved": round(model / (kernel_ns * 1e-9) / 1e9, 2), "peak": 8000.0, "unit": "GB/s"}
    out["frac"] = round(out["achieved"] / out["peak"], 4)
    traffic = {}
    for sub, name in (("bnbs_pmc_fetch", "FETCH_SIZE"), ("bnbs_pmc_write", "WRITE_SIZE")):
        dp = os.path.join(ROOT, "profiles", f"{tag}_{sub}")
        if profile_matches(dp) != "library":
            return out
        c2 = _exact_cum(os.path.join(dp, "exact_cum.log"))
        kb = 0.0
        for path in glob.glob(os.path.join(dp, "*counter_collection.csv")):
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                        kb += float(r["Counter_Value"])
        if not c2 or not c2[0] or not kb:
            return out
        traffic[name] = kb * 1024.0 * (FETCH_CORRECTION if name == "FETCH_SIZE" else 1.0) / c2[0]
    per_block = traffic["FETCH_SIZE"] + traffic["WRITE_SIZE"]
    out["traffic_bytes_per_pass_block"] = round(per_block, 1)
    out["model_bytes_per_pass_block"] = round(model / blocks, 1)
    out["traffic"] = round(per_block * blocks, 1)
    out["traffic_source"] = (f"profiles/{tag}_bnbs_pmc_fetch / _write (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                             f"FETCH_SIZE x {FETCH_CORRECTION}), per pass-block of each run's own counters")
    return out


def sub_profile_block(tag: str):
    """Issue / LDS counters of the subproblem kernel alone (tools/sub_bench.py, C4 32 paths x 256
    scenarios, cold: the bench's subproblem leg), from profiles/<tag>_sub_pmc when collected with
    this very library; else None.  The pass counts per scenario of the B&B legs are in
    profiles/<tag>_sub_pass_counts.txt."""
    import csv
    dp = os.path.join(ROOT, "profiles", f"{tag}_sub_pmc")
    if profile_matches(dp) != "library":
        return None
    c = {}
    for path in glob.glob(os.path.join(dp, "*counter_collection.csv")):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                if "k_sub_scenario" in r["Kernel_Name"]:
                    c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    wc = c.get("SQ_WAVE_CYCLES")
    if not wc:
        return None
    insts = c.get("SQ_INSTS_VALU", 0.0) + c.get("SQ_INSTS_SALU", 0.0)
    return {"source": f"profiles/{tag}_sub_pmc (rocprofv3 --pmc SQ_* of tools/sub_bench.py --cfg C4 --scenarios 256 "
                      f"--paths 32 --reps 3, libsgufp_hip.so sha256 {lib_sha256()[:16]}; wave cycles in quad-cycles)",
            "active_frac": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
            "wait_frac": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 4),
            "lds_active_frac": round(c.get("SQ_ACTIVE_INST_LDS", 0.0) / wc, 4),
            "lds_bank_conflict_frac": round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, c.get("SQ_ACTIVE_INST_LDS", 0.0)), 4),
            "cycles_per_wave_instruction": round(4.0 * wc / max(1.0, insts), 2),
            "pass_counts": f"profiles/{tag}_sub_pass_counts.txt"}


def _native_comm(eng, world, rank):
    """The library's own RCCL communicator (shard.cpp) on this rank's context: the id made on
    rank 0 reaches the others through a gloo side group (plain bytes)."""
    import torch
    import torch.distributed as dist
    from sgufp_solver_amd import engine as E
    side = dist.new_group(backend="gloo")
    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        uid[:] = torch.frombuffer(bytearray(E.comm_unique_id()), dtype=torch.uint8)
    dist.broadcast(uid, src=0, group=side)
    eng.comm_init(world, rank, bytes(uid.numpy()))


def bnb_run(cfg_name, seed, lb_mode, budget, batch, round_seconds, work, device=0, progress=10.0, tag="bnb",
            heuristic=0, streams=1, native=False):
    """The device DDSolver (sgufp_bnb_step rounds) from the root record Node{} with no
    incumbent, after a short warm-up search (kernels, allocations; its pool is cleared):
    relaxations = NodeExplorer::process calls, exact-leaf refinement loops with the device
    subproblem included; a round's loops stop after round_seconds (deferred, resumed later).
    heuristic > 0: the incumbent is seeded inside the timed region by the restricted-DD
    heuristic of that width on the root record (processX3's restricted half, restricted.py),
    as the reference seeds it with a known value (main.cpp:75), so incumbent pruning acts.
    streams > 1: that many frontier shards on the device, one context (HIP stream, scratch)
    and one host thread each, exchanging as the multi-rank shards do (shards.LocalComm).
    With torch.distributed initialised (N ranks, one GPU each) the search is shared by the N
    shards (strong scaling): native=True runs the round exchanges through the library's own
    RCCL communicator (shard.cpp: incumbent all-reduce, cut-row all-gather, frontier sizes,
    ncclSend / ncclRecv work sharing), else through shards.py over the torch group."""
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MIN
    from sgufp_solver_amd.solver import DDSolver
    cfg = instance.CONFIGS[cfg_name]
    inst = instance.generate(cfg, seed)
    if lb_mode == "zero":
        inst.lb[:] = 0
    net = os.path.join(work, f"{tag}_{cfg_name}.txt")
    inst.write(net)
    from sgufp_solver_amd.shards import LocalComm, LocalGroup, run_local_shards
    import torch
    dist_world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    dist_rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    native = native and dist_world > 1
    group = LocalGroup(streams) if streams > 1 else None
    solvers = [DDSolver(net, device=device, max_batch=batch, verbose=False, time_budget=2.0, progress=progress,
                        round_seconds=min(round_seconds, 2.0), comm=LocalComm(group, k) if group else None,
                        native_world=dist_world if native else 0)
               for k in range(streams)]
    if native:
        _native_comm(solvers[0].eng, dist_world, dist_rank)
    run_local_shards(solvers, lambda s: s.start_solver(DOUBLE_MIN))       # warm-up
    for s in solvers:
        s.eng.clear_cuts()
        s.eng.set_timing(True)
        s.time_budget = budget
        s.round_seconds = round_seconds
        s.restricted_width = heuristic
    solver = solvers[0]
    if native:
        solver.eng.cuts_exchange()      # the warm-up's marks: nothing left to send
        solver.eng.incumbent_allreduce(0.0)   # a collective as a barrier on the library's stream
    elif solver.shard_comm is not None and group is None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    z = run_local_shards(solvers, lambda s: s.start_solver(DOUBLE_MIN))[0]
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    c = {k: sum(int(s.counters[k]) for s in solvers) for k in solver.counters}
    world = 1
    keys = sorted(c)
    if native:
        world = dist_world
        vals = [int(c[k]) for k in keys] + [int(elapsed * 1e6), int(solver.received)]
        cols = [solver.eng.comm_allgather_i64(vals[i:i + 4], world) for i in range(0, len(vals), 4)]
        g = np.concatenate(cols, axis=1)
        c = {k: int(v) for k, v in zip(keys, g[:, :len(keys)].sum(axis=0))}
        elapsed = float(g[:, len(keys)].max()) / 1e6
        received = [int(x) for x in g[:, len(keys) + 1]]
    elif solver.shard_comm is not None and group is None:
        comm = solver.shard_comm
        world = comm.world
        g = comm.allgather_i64([int(c[k]) for k in keys] + [int(elapsed * 1e6), int(solver.received)])
        c = {k: int(v) for k, v in zip(keys, g[:, :len(keys)].sum(axis=0))}
        elapsed = float(g[:, len(keys)].max()) / 1e6
        received = [int(x) for x in g[:, len(keys) + 1]]
    else:
        received = [int(s.received) for s in solvers]
    out = {
        "workload": f"{cfg_name}: {cfg.n_arcs}-arc layered network, {inst.scenarios} scenarios"
                    f"{' (lower bounds 0)' if lb_mode == 'zero' else ''}, root record, "
                    f"{f'incumbent seeded by the width-{heuristic} restricted-DD heuristic' if heuristic else 'no incumbent'}, "
                    f"{f'{streams} frontier shards on the device (one stream and host thread each), ' if streams > 1 else ''}"
                    f"up to {batch} records per round, refinement loops deferred after {round_seconds} s per round",
        "instance_seed": seed, "total_layers": int(solver.eng.info.total_layers), "n_gpus": world,
        "relaxations_per_s": round(c["relaxed"] / elapsed, 2),
        "subproblems_per_s": round(c["subproblems"] / elapsed, 2),
        "scenario_lps_per_s": round(c["subproblems"] * inst.scenarios / elapsed, 1),
        "cuts_generated": int(c["new_feasibility_cuts"] + c["new_optimality_cuts"]),
        "seconds": round(elapsed, 3), "rounds": solver.rounds, "complete": all(s.complete for s in solvers),
        "incumbent": z, "streams": streams,
        "heuristic_incumbent": solver.heuristic_incumbent,
        "frontier_left": sum(s.eng.frontier_size() for s in solvers),
        "pool": [solver.eng.cuts_count(1), solver.eng.cuts_count(0)], "counters": c,
    }
    if world > 1:
        out["exchange"] = ("library RCCL communicator (shard.cpp: ncclAllReduce / ncclAllGather / ncclSend+Recv)"
                           if native else f"shards.py over torch.distributed ({torch.distributed.get_backend()})")
        out["records_received_per_rank"] = received
    for s in solvers:
        s.eng.close()
    return out


def bnb_main(args):
    """Full B&B on the device (BASELINE configs[2]: 1k-arc network, 64 scenarios) for
    --bnb-seconds; with N ranks the search is shared (incumbent all-reduce, cut all-gather,
    work sharing: strong scaling)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = dist_backend(torch)
        if torch.cuda.is_available():
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend)
    heartbeat("bnb", 20.0)
    work = tempfile.mkdtemp(prefix=f"sgufp_bnb_r{rank}_")
    out = bnb_run(args.bnb_config, args.seed, args.bnb_lb, args.bnb_seconds, args.nodes, args.round_seconds, work,
                  heuristic=args.bnb_heuristic, streams=args.bnb_streams,
                  device=local % max(1, torch.cuda.device_count()))
    line = {"metric": "device B&B: node relaxations/s (NodeExplorer::process incl. exact-leaf subproblems)",
            "value": out["relaxations_per_s"], "unit": "relaxations/s", "n_gpus": world,
            "higher_is_better": True, "scaling": "strong", "dtype": "f64", "data": "synthetic", **out}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def dist_backend(torch) -> str:
    """RCCL ("nccl") between GPUs; SGUFP_BENCH_BACKEND=gloo rehearses the multi-rank protocol
    with several ranks on one card (RCCL refuses two ranks on one device)."""
    return os.environ.get("SGUFP_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")


def heartbeat(tag="bench", every=30.0):
    """A progress line on stderr while the legs run (long phases print nothing else)."""
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(every)
            print(f"[{tag}] running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    if args.mode == "bnb":
        return bnb_main(args)
    heartbeat()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = dist_backend(torch)
        if torch.cuda.is_available():
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
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
    eng = E.Engine(net, local % max(1, torch.cuda.device_count()), max(n, 1024))
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

    # With N ranks every step is one B&B round of a frontier shard: the relaxation of its
    # records, then the round's exchanges over RCCL (sgufp_solver_amd/shards.py) -- the
    # incumbent all-reduce(MAX) and the all-gather of the cut rows the round appended (a
    # DD-only step closes no exact leaf and adds no rows: the collectives still run).
    comm = None
    marks = {1: eng.cuts_count(1), 0: eng.cuts_count(0)}
    if dist:
        from sgufp_solver_amd.shards import ShardComm
        comm = ShardComm()

    def step(z):
        eng.relax_async(z)
        eng.sync()
        if comm is not None:
            z = comm.allreduce_max(z)
            comm.exchange_cuts(eng, marks)
        return z

    eng.set_timing(True)
    for _ in range(args.warmup):
        step(incumbent)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    relax_ms = []
    emit_ms = []
    bytes0 = comm.bytes if comm else 0
    t0 = time.perf_counter()
    z = incumbent
    for _ in range(args.steps):
        z = step(incumbent)
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

    # per-launch SURVEY 8(d) byte model: 6A + sum_cuts(14A + 8N) + record in
    st, ex, lb, ub, nc = eng.results_arrays()
    dn, da, dl, sw = eng.stats()
    g = mine.gl.astype(np.float64)
    ns = np.diff(mine.states_off).astype(np.float64)
    r_in = 2 * g + 2 * ns + 24
    bytes_model = float(np.sum(6.0 * da + sw * (14.0 * da + 8.0 * dn) + r_in))
    ch = eng.children_batch()
    r_out = float(np.sum(2 * ch.gl.astype(np.float64) + 2 * np.diff(ch.states_off) + 24)) if ch.n else 0.0
    t_relax = float(np.mean(relax_ms)) / 1e3
    model_gbps = bytes_model / t_relax / 1e9
    traffic, traffic_src = pmc_traffic(args.profile_tag, workload_key(args))
    achieved = traffic / t_relax / 1e9 if traffic else None

    total_nodes = mine.n * world
    value = total_nodes * args.steps / elapsed
    gpu_sample = None
    if rank == 0 and world == 1 and not args.no_cpu:
        k = min(args.cpu_sample, mine.n)
        gpu_sample = eng._collect()[:k]          # the last timed step's results, record order
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
            "parallelism": f"frontier shards x{world}" + (", per-step incumbent all-reduce + cut-row all-gather"
                                                          if world > 1 else ""),
        },
        "roofline": {
            # the roofline that bounds this class of kernel (no MFMA work): HBM.  achieved /
            # frac are the HBM bytes the counters measured for this build (FETCH_SIZE x 2 +
            # WRITE_SIZE per launch) over the launch time; the SURVEY 8(d) byte model counts
            # every (arc, cut) operand as if streamed from HBM, which the kernel serves from LDS
            # / L2 -- reported separately as model_gbps, it is not HBM traffic.
            "bound": "hbm",
            "limiter": "latency/issue (DESIGN.md section 5: issue counters in profiles/)",
            "kernel": "k_relax",
            "achieved": round(achieved, 2) if achieved else None,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "avg_launch_ms": round(t_relax * 1e3, 4),
            "emit_ms": round(float(np.mean(emit_ms)), 4),
            "issue": pmc_issue(args.profile_tag, workload_key(args)),
            "model_gbps": round(model_gbps, 2),
            "model_bytes_per_launch": bytes_model,
            "model": "SURVEY 8(d): 6A + sum over applied cuts (14A + 8N) + records (A, N, cuts counted per record)",
            "children_record_bytes": r_out,
        },
        "cpu_baseline": None,
        "parity": None,
        "subproblem": sub,
    }
    if comm is not None:
        line["exchange_bytes_per_step"] = round((comm.bytes - bytes0) / args.steps, 1)
    if rank == 0 and world == 1 and not args.no_cpu:
        cb, par = cpu_baseline(work, net, pool, mine, incumbent, args, gpu_sample)
        line["cpu_baseline"] = cb
        line["parity"] = par
        if sub is not None:
            i0, n0 = sub["_inst0"]
            sub["cpu_baseline"] = cpu_subproblem_baseline(inst, net, sub["_paths"], args, i0, n0)
    if sub is not None:
        sub.pop("_paths", None)
        sub.pop("_inst0", None)
        sub["counters"] = sub_profile_block(args.profile_tag)
    eng.close()
    if rank == 0 and world == 1 and args.bnb_leg_seconds > 0:
        # BASELINE metric with the subproblems in the loop: the device B&B on the same
        # 1k-arc network with its 256 scenarios (lower bounds 0: feasible, optimality cuts)
        line["bnb"] = bnb_run(args.config, args.seed, "zero", args.bnb_leg_seconds, 1024, args.round_seconds, work,
                              device=local, progress=0.0, tag="leg")
        if args.bnb_seeded_width > 0:
            # the same search with incumbent pruning acting (BASELINE configs[2]): the incumbent
            # seeded inside the timed region by the restricted-DD heuristic on the root record
            line["bnb_seeded"] = bnb_run(args.config, args.seed, "zero", args.bnb_leg_seconds, 1024,
                                         args.round_seconds, work, device=local, progress=0.0, tag="legs",
                                         heuristic=args.bnb_seeded_width)
            line["bnb_seeded"]["roofline"] = bnb_profile_block(args.profile_tag)
            if args.cpp_leg_seconds > 0:
                # the same seeded search through the C++ host path a maintainer links
                line["bnb_seeded_cpp"] = cpp_bnb_run(args.config, args.seed, "zero", args.cpp_leg_seconds, 1024,
                                                     args.round_seconds, args.bnb_seeded_width, work)
        if args.bnb_gen_seconds > 0 and args.bnb_seeded_width > 0:
            # the instance as generated (sink-arc lower bounds kept): infeasible scenarios, the
            # first one's ray as a feasibility cut (grb.cpp:284-351) in the loop
            line["bnb_gen"] = bnb_run(args.config, args.seed, "gen", args.bnb_gen_seconds, 1024, args.round_seconds,
                                      work, device=local, progress=0.0, tag="legg", heuristic=args.bnb_seeded_width)
    if rank == 0 and world == 1 and args.bnb_parity_rounds > 0:
        line["bnb_parity"] = bnb_parity_leg(args)
    if rank == 0 and world == 1 and args.config == "C4" and args.c5_nodes > 0:
        line["config5"] = config5_leg(args, work)
    if world > 1 and args.bnb_leg_seconds > 0:
        # BASELINE configs[3]: one search shared by the N frontier shards (strong scaling), the
        # round exchanges over the library's own RCCL communicator -- beside the weak-scaling
        # relaxation step above.  A watchdog prints the line without this leg should a shard
        # stall in a collective.
        guarded_leg(line, "bnb_multi", lambda: bnb_run(
            args.config, args.seed, "zero", args.bnb_leg_seconds, 1024, args.round_seconds, work,
            device=local % max(1, torch.cuda.device_count()), progress=0.0, tag="multi",
            heuristic=args.bnb_seeded_width, native=dist_backend(torch) == "nccl"),
            rank, args.bnb_leg_seconds + 240.0)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


WATCHDOG_EXIT = 3   # a stalled collective fails the run (exit status), it is not hidden in the line


def watchdog(seconds, line, rank):
    """After `seconds` without stop.set(): rank 0 prints the line built so far (the leg marked
    as timed out) and every rank exits with WATCHDOG_EXIT (a shard stuck in a collective cannot
    be unwound, and a run that stalled must not look like a successful one)."""
    import threading
    stop = threading.Event()

    def run():
        if not stop.wait(seconds):
            if rank == 0:
                line["bnb_multi"] = {"error": f"timed out after {seconds:.0f} s"}
                print(json.dumps(line), flush=True)
            sys.stdout.flush()
            sys.stderr.write(f"bench: rank {rank}: multi-rank leg stalled for {seconds:.0f} s, exiting {WATCHDOG_EXIT}\n")
            sys.stderr.flush()
            os._exit(WATCHDOG_EXIT)

    threading.Thread(target=run, daemon=True).start()
    return stop


LEG_FAIL_EXIT = 4   # a multi-rank leg that raised on any rank fails the run on every rank


def guarded_leg(line, key, run, rank, seconds):
    """line[key] = run() on every rank of a multi-rank job, under the watchdog.  A rank whose
    run raises records the error in the line; then every rank learns of it through a gloo
    all-reduce of the failure flags (so a rank that finished cleanly does not exit 0 beside a
    failed one), rank 0 prints the line, and every rank exits LEG_FAIL_EXIT.  A rank stuck in a
    collective the failed one never joins is ended by the watchdog (WATCHDOG_EXIT)."""
    import torch
    import torch.distributed as dist
    stop = watchdog(seconds, line, rank)
    failed = 0
    try:
        line[key] = run()
    except Exception as e:     # noqa: BLE001 -- the error goes into the line, then the run fails
        line[key] = {"error": f"{type(e).__name__}: {e}"}
        failed = 1
        sys.stderr.write(f"bench: rank {rank}: {key} failed: {type(e).__name__}: {e}\n")
    flag = torch.tensor([failed], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=dist.new_group(backend="gloo"))
    stop.set()
    if int(flag.item()):
        if rank == 0:
            if not failed:
                line[key] = {"error": "failed on another rank", "partial": line.get(key)}
            print(json.dumps(line), flush=True)
        sys.stdout.flush()
        sys.stderr.write(f"bench: rank {rank}: multi-rank leg {key} failed, exiting {LEG_FAIL_EXIT}\n")
        sys.stderr.flush()
        os._exit(LEG_FAIL_EXIT)


def cpp_bnb_run(cfg_name, seed, lb_mode, budget, batch, round_seconds, width, work):
    """bnb_run's search through the C++ host API instead of the Python driver:
    Inavap::DDSolver (include/sgufp/inavap.hpp) with restricted-DD seeding and a time budget,
    driven by tests/host/host_api_test "search" (warm-up of 2 s, pool dropped, then the timed
    search from the root record)."""
    import subprocess
    from sgufp_solver_amd import instance
    cfg = instance.CONFIGS[cfg_name]
    inst = instance.generate(cfg, seed)
    if lb_mode == "zero":
        inst.lb[:] = 0
    net = os.path.join(work, f"cpp_{cfg_name}.txt")
    inst.write(net)
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sgufp_solver_amd", "lib", "host_api_test")
    r = subprocess.run([exe, "search", net, str(width), str(budget), str(batch), str(round_seconds), "0", "0"],
                       capture_output=True, text=True, timeout=budget + 300)
    if r.returncode != 0:
        raise RuntimeError(f"host_api_test search failed: {r.stderr[-1000:]}")
    out = {"counters": {}}
    for ln in r.stdout.splitlines():
        p = ln.split()
        if p and p[0] == "search":
            out.update(incumbent=float.fromhex(p[1]), heuristic_incumbent=float.fromhex(p[2]), seconds=float(p[3]),
                       rounds=int(p[4]), complete=p[5] == "1")
        elif p and p[0] == "counter":
            out["counters"][p[1]] = int(p[2])
        elif p and p[0] == "pool":
            out["pool"] = [int(p[1]), int(p[2])]
    c, sec = out["counters"], out["seconds"]
    out["relaxations_per_s"] = round(c["relaxed"] / sec, 2)
    out["subproblems_per_s"] = round(c["subproblems"] / sec, 2)
    out["scenario_lps_per_s"] = round(c["subproblems"] * inst.scenarios / sec, 1)
    out["workload"] = (f"{cfg_name}: {cfg.n_arcs}-arc layered network, {inst.scenarios} scenarios"
                       f"{' (lower bounds 0)' if lb_mode == 'zero' else ''}, root record, incumbent seeded by the "
                       f"width-{width} restricted-DD heuristic, up to {batch} records per round, refinement loops "
                       f"deferred after {round_seconds} s per round; C++ Inavap::DDSolver (libsgufp_host.so)")
    return out


def bnb_parity_leg(args):
    """The device B&B under the cuts its own subproblem makes, checked round by round against
    the reference (oracle/bnb_parity.check_search: the popped records vs ref_dd relaxp bit for
    bit, bound pruning, cut tightness, closed-loop bounds vs the matchings' expected values and
    HiGHS, one refinement loop vs ref_dd refine) on the bench network, seeded."""
    from oracle import bnb_parity as bp
    if not os.path.exists(bp.REF_BIN):
        return None
    # at the pool size the timed legs run against: the seeded search until 10^4 optimality
    # cuts, then the next round's batch (exact records, non-exact records a cut prunes)
    rep = bp.check_large_pool(args.config, args.seed, args.bnb_seeded_width, min_opt_cuts=args.bnb_parity_pool,
                              per_kind=6)
    fails = rep.pop("failures")
    rep["pool_last"] = rep["pool_total"]
    rep["against"] = ("oracle/_ref/ref_dd (the reference's RelaxedDDNew) relaxp on the pool and next batch of the "
                      "running device search")
    if args.bnb_parity_survivor_pool > 0:
        # the unseeded search (every non-exact record survives every cut): survivors the
        # cut-parallel non-exact phase settled (k_nx_dag / k_exact_leaf<nx> / k_nx_fin), with
        # their cutset children, against relaxp
        sv = bp.check_nx_survivors(args.config, args.seed, (args.bnb_parity_survivor_pool,), per_pool=8)
        fails += sv.pop("failures")
        rep["survivors"] = sv
        rep["sampled"]["survivor"] += sum(p["survivors_checked"] for p in sv["pools"])
        rep["checked"] += sum(p["checked"] for p in sv["pools"])
        rep["mismatches"] += sum(p["mismatches"] for p in sv["pools"])
    if args.bnb_parity_rounds > 0:
        # round by round at small pools: the popped records, bound pruning, cut tightness, one
        # refinement loop replayed against ref_dd refine
        cs = bp.check_search(args.config, args.seed, args.bnb_seeded_width, rounds=40, batch=64, sample=16,
                             min_subproblems=1, rounds_after=args.bnb_parity_rounds, round_iters=2)
        fails += cs.pop("failures")
        rep["search"] = {k: cs[k] for k in ("rounds", "checked", "mismatches", "subproblems", "opt_cuts", "feas_cuts",
                                            "replayed", "pool_last", "seconds")}
    rep["bit_exact"] = not fails and rep["mismatches"] == 0
    rep["first_failures"] = fails[:5]
    return rep


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
    parity = None
    if not args.no_parity and args.c5_parity > 0:
        # the last timed step's first records against the reference's RelaxedDDNew
        k = min(args.c5_parity, fr.n)
        got = eng._collect()[:k]
        sample = E.batch_slice(fr, np.arange(k))
        nodes, cuts, outp = (os.path.join(work, f) for f in ("c5_nodes.txt", "c5_cuts.txt", "c5_ref.txt"))
        pools.write_nodes(nodes, E.batch_to_records(sample))
        pools.write_pool(cuts, pool)
        ref = os.path.join(ROOT, "oracle", "_ref", "ref_dd")
        if os.path.exists(ref):
            r = subprocess.run([ref, "relaxp", net, cuts, nodes, inc.hex(), "16", outp], capture_output=True, text=True,
                               timeout=900)
            if r.returncode == 0:
                bad, msgs = compare_results(got, pools.read_results(outp))
                parity = {"checked": k, "mismatches": bad, "bit_exact": bad == 0, "first_mismatches": msgs,
                          "against": "oracle/_ref/ref_dd relaxp (the reference's RelaxedDDNew), same records, pool "
                                     "and incumbent", "ref_seconds": json.loads(r.stdout.strip().splitlines()[-1])["seconds"]}
    out = {"workload": f"C5: {cfg.n_arcs}-arc layered network, {inst.scenarios} scenarios, {args.n_feas}F+{args.n_opt}O "
                       f"pool, BFS frontier of {fr.n} open nodes", "instance_seed": args.seed, "incumbent": inc,
           "relaxations_per_s": round(fr.n * steps / wall, 2), "k_relax_ms": round(float(np.mean(ms)), 4),
           "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
           "avg_dd_nodes": float(np.mean(dn)), "avg_sweeps": float(np.mean(sw)), "parity": parity}
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
    if args.c5_bnb_seconds > 0:
        # BASELINE configs[4]: the device B&B with cut generation in the loop (exact leaves
        # call the 512-scenario subproblem, new cuts join the pool every refinement step)
        out["bnb"] = bnb_run("C5", args.seed, "zero", args.c5_bnb_seconds, 1024, args.round_seconds, work,
                             progress=0.0, tag="c5leg")
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


def _bits(x: float) -> int:
    import struct
    return struct.unpack("<q", struct.pack("<d", x))[0]


def compare_results(got, want):
    """Bit-exact comparison of NodeExplorer::process outcomes (status, exact flag, lb / ub
    bit patterns, argmax path of exact DDs, cutset children -- the branching indices --, DD
    sizes); returns (number of records that differ, first messages)."""
    def key(nd):
        return (nd.gl, _bits(nd.lb), _bits(nd.ub), tuple(nd.states), tuple(nd.sol))
    bad, msgs = 0, []
    for k, (g, w) in enumerate(zip(got, want)):
        why = None
        if g.status != w.status or g.exact != w.exact:
            why = f"status/exact {(g.status, g.exact)} != {(w.status, w.exact)}"
        elif _bits(g.lb) != _bits(w.lb) or _bits(g.ub) != _bits(w.ub):
            why = f"bounds {(g.lb, g.ub)} != {(w.lb, w.ub)}"
        elif g.path != w.path:
            why = "argmax path differs"
        elif [key(c) for c in g.children] != [key(c) for c in w.children]:
            why = f"children differ ({len(g.children)} vs {len(w.children)})"
        elif (g.dd_nodes, g.dd_arcs, g.dd_layers) != (w.dd_nodes, w.dd_arcs, w.dd_layers):
            why = "DD size differs"
        if why:
            bad += 1
            if len(msgs) < 5:
                msgs.append(f"record {k}: {why}")
    if len(got) != len(want):
        bad += abs(len(got) - len(want))
        msgs.append(f"{len(got)} results vs {len(want)}")
    return bad, msgs


def cpu_baseline(work, net, pool, batch, incumbent, args, gpu_sample=None):
    """The reference's own RelaxedDDNew (oracle/_ref/ref_dd, built from its sources) on the
    host cores over a bounded sample of the same frontier (same pool and incumbent): every
    record of the sample, a work queue over the threads ("relaxp").  Its outputs are also
    the parity check of the timed workload: the GPU results of the last timed step for the
    same records must equal them bit for bit.  Falls back to the clean-room port's timing
    (no parity) when the reference build is absent.  Returns (cpu_baseline, parity)."""
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import pools
    sample = E.batch_slice(batch, np.arange(min(args.cpu_sample, batch.n)))
    nodes = os.path.join(work, "nodes.txt")
    cuts = os.path.join(work, "cuts.txt")
    pools.write_nodes(nodes, E.batch_to_records(sample))
    pools.write_pool(cuts, pool)
    # every host core (std::thread::hardware_concurrency()), and the job's CPU
    # quota (cgroup cpu.max) when that is smaller: on the GPU box os.cpu_count() shows the whole
    # machine while this job may run 16 CPUs, so the quota-sized run is faster; the faster of the
    # two is the baseline and both are reported
    threads = max(1, os.cpu_count() or 1)
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = threads
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(round(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
    except Exception:
        pass
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_dd")
    if os.path.exists(ref):
        out_path = os.path.join(work, "ref_results.txt")
        r = subprocess.run([ref, "relaxp", net, cuts, nodes, incumbent.hex(), str(threads), out_path],
                           capture_output=True, text=True, timeout=600)
        if r.returncode == 0:
            out = json.loads(r.stdout.strip().splitlines()[-1])
            cb = {"value": round(out["relaxations"] / out["seconds"], 2), "unit": "relaxations/s", "cores": threads,
                  "kind": "reference", "cpu": cpu_model, "cpus_allowed": allowed,
                  "sample": f"the first {sample.n} open nodes of the timed frontier, same pool and incumbent, "
                            f"{out['seconds']:.1f} s on {threads} threads (os.cpu_count())"}
            cb["value_all_threads"] = cb["value"]
            cb["cpu_quota"] = quota
            alt = min(quota or 16, threads)
            if alt != threads:
                r2 = subprocess.run([ref, "relaxp", net, cuts, nodes, incumbent.hex(), str(alt),
                                     os.path.join(work, "ref_results_q.txt")], capture_output=True, text=True,
                                    timeout=600)
                if r2.returncode == 0:
                    o2 = json.loads(r2.stdout.strip().splitlines()[-1])
                    v2 = round(o2["relaxations"] / o2["seconds"], 2)
                    cb[f"value_{alt}_threads"] = v2
                    if v2 > cb["value"]:
                        cb["value"], cb["cores"] = v2, alt
                        cb["sample"] = (f"the first {sample.n} open nodes of the timed frontier, same pool and "
                                        f"incumbent, {o2['seconds']:.1f} s on {alt} threads (the job's CPU share; "
                                        f"{threads} threads = os.cpu_count(): {cb['value_all_threads']}/s)")
            parity = None
            if gpu_sample is not None and not args.no_parity:
                want = pools.read_results(out_path)
                bad, msgs = compare_results(gpu_sample, want)
                parity = {"checked": len(want), "mismatches": bad, "bit_exact": bad == 0,
                          "against": "oracle/_ref/ref_dd relaxp (the reference's RelaxedDDNew) on the same records, "
                                     "pool and incumbent",
                          "fields": "status, exact, lb/ub bits, argmax path, cutset children, DD sizes",
                          "first_mismatches": msgs}
            return cb, parity
    exe = os.path.join(ROOT, "oracle", "_build", "dd_oracle")
    if os.path.exists(exe):
        r = subprocess.run([exe, "time", net, cuts, nodes, incumbent.hex(), str(threads), str(args.cpu_seconds)],
                           capture_output=True, text=True, timeout=args.cpu_seconds * 4 + 120)
        if r.returncode == 0:
            out = json.loads(r.stdout.strip().splitlines()[-1])
            return ({"value": round(out["relaxations"] / out["seconds"], 2), "unit": "relaxations/s", "cores": threads,
                     "kind": "port", "cpu": cpu_model,
                     "sample": f"{out['relaxations']} of the first {sample.n} open nodes of the same frontier, same "
                               f"pool and incumbent, {out['seconds']:.1f} s on {threads} threads"}, None)
    return None, None


if __name__ == "__main__":
    main()
