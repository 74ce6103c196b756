"""Per-node diagnostics of one relaxation step on the bench workload (GPU).

    python tools/relax_diag.py [--config C4 --seed 1 --nodes 4096 --cb 16]

Prints the k_relax time, the distribution of per-wave wall-clock ticks against DD
size / status / cuts applied / batched-sweep restarts."""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--cb", default=None)
    ap.add_argument("--incumbent", default="p40")
    args = ap.parse_args()
    if args.cb:
        os.environ["SGUFP_CUT_BATCH"] = args.cb
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import frontier, instance, pools
    inst = instance.generate(instance.CONFIGS[args.config], args.seed, scenarios=1)
    d = tempfile.mkdtemp()
    inst.write(f"{d}/net.txt")
    eng = E.Engine(f"{d}/net.txt", 0, args.nodes)
    fr = frontier.bfs_frontier(eng, args.nodes)
    eng.add_cuts(pools.synthetic_pool(inst, 16, 64, args.seed))
    eng.upload(fr)
    if args.incumbent.startswith("p"):
        eng.relax_async(pools.DOUBLE_MIN)
        eng.sync()
        st, ex, lb, ub, nc = eng.results_arrays()
        inc = float(np.percentile(ub[(st == 0) | (st == 3)], float(args.incumbent[1:])))
    else:
        inc = float(args.incumbent)
    eng.set_timing(True)
    for _ in range(2):
        eng.relax_async(inc)
        eng.sync()
    t0 = time.perf_counter()
    eng.relax_async(inc)
    eng.sync()
    wall = time.perf_counter() - t0
    ms_relax, ms_emit = eng.last_timing()
    st, ex, lb, ub, nc = eng.results_arrays()
    dn, da, dl, sw = eng.stats()
    ticks, rinfo = eng.debug()
    rinfo = rinfo.astype(np.int64) & 0xFFFFFFFF
    redo = rinfo & 0xFF
    stream = (rinfo >> 31) & 1
    mirsz = (rinfo >> 8) & 0x7FFFFF
    us = ticks / 100.0
    print(f"cb={os.environ.get('SGUFP_CUT_BATCH', 'default')} inc={inc:.3f} k_relax={ms_relax:.2f} ms "
          f"emit={ms_emit:.3f} ms wall={wall * 1e3:.2f} ms")
    print(f"status {dict(zip(*np.unique(st, return_counts=True)))} exact={int(ex.sum())}")
    print(f"wave us: mean {us.mean():.1f} p50 {np.median(us):.1f} p90 {np.percentile(us, 90):.1f} "
          f"max {us.max():.1f}; sum/CU(256) {us.sum() / 256 / 1e3:.2f} ms")
    print(f"dd nodes mean {dn.mean():.0f} max {dn.max()}; sweeps mean {sw.mean():.1f}; redo mean {redo.mean():.2f} "
          f"max {redo.max()}; stream {stream.mean():.2f} (entries mean {mirsz.mean():.0f} max {mirsz.max()}) "
          f"cap {eng.info.node_capacity}")
    for s in np.unique(st):
        m = st == s
        print(f"  status {s}: n={m.sum()} us/node {us[m].mean():.1f} sweeps {sw[m].mean():.1f} "
              f"us/sweep {np.mean(us[m] / np.maximum(sw[m], 1)):.2f} redo {redo[m].mean():.2f}")
    ph = eng.phases() / 100.0
    names = ["build", "narrow", "tail", "last", "post", "redo", "finish", "epilog"]
    print("phase us/node: " + ", ".join(f"{nm} {ph[:, k].mean():.0f}" for k, nm in enumerate(names)))
    big = np.argsort(-us)[:5]
    for k in big:
        print(f"  slow node {k}: {us[k]:.0f} us, dd {dn[k]} nodes, {dl[k]} layers, sweeps {sw[k]}, status {st[k]}, "
              f"redo {redo[k]}")


if __name__ == "__main__":
    main()
