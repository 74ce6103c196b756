"""ctypes binding of libsgufp_hip.so (include/sgufp_hip.h).

The Python side is plumbing for tests, the bench and the multi-GPU driver; the
relaxation itself runs in the HIP kernels.  There is deliberately no CPU fallback:
if the library cannot be loaded the constructor raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .pools import NodeRecord, PoolCut, RelaxResult

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SGUFP_LIB_PATH") or os.path.join(HERE, "lib", "libsgufp_hip.so")

SUCCESS, PRUNED_F, PRUNED_O, NEEDS_SUBPROBLEM, PRUNED_BOUND = 0, 1, 2, 3, 4
# sgufp_batch_routes (include/sgufp_hip.h)
ROUTE_IN_ORDER, ROUTE_EXACT_PHASE, ROUTE_NX_PHASE, ROUTE_NX_FALLBACK = 0, 1, 2, 3
ERR_RECORD, ERR_CAPACITY, ERR_CUTSET = 16, 17, 18

EXPORTS = [
    "sgufp_create_from_file", "sgufp_create", "sgufp_destroy", "sgufp_get_network_info",
    "sgufp_processing_order", "sgufp_last_error", "sgufp_stream", "sgufp_cuts_append",
    "sgufp_cuts_clear", "sgufp_cuts_count", "sgufp_batch_upload", "sgufp_batch_relax",
    "sgufp_batch_sync", "sgufp_batch_results", "sgufp_batch_children_size", "sgufp_batch_children",
    "sgufp_batch_paths", "sgufp_batch_stats", "sgufp_batch_refine", "sgufp_set_timing",
    "sgufp_last_timing", "sgufp_probe_network", "sgufp_batch_debug",
    "sgufp_batch_phases", "sgufp_subproblem", "sgufp_subproblem_detail", "sgufp_slot_keys",
    "sgufp_cuts_append_rows", "sgufp_frontier_clear", "sgufp_frontier_size", "sgufp_frontier_push",
    "sgufp_frontier_take_size", "sgufp_frontier_take", "sgufp_bnb_step", "sgufp_cuts_rows",
    "sgufp_restricted_relax", "sgufp_restricted_results", "sgufp_restricted_paths", "sgufp_restricted_cutset_size",
    "sgufp_restricted_cutset", "sgufp_bnb_set_limits", "sgufp_comm_unique_id", "sgufp_comm_init",
    "sgufp_comm_info", "sgufp_comm_destroy", "sgufp_incumbent_allreduce", "sgufp_cuts_exchange",
    "sgufp_frontier_sizes", "sgufp_frontier_balance", "sgufp_bnb_set_trace", "sgufp_bnb_trace",
    "sgufp_frontier_peek_size", "sgufp_frontier_peek", "sgufp_balance_plan", "sgufp_comm_allgather_i64",
    "sgufp_dd_build", "sgufp_dd_apply", "sgufp_dd_solution", "sgufp_dd_cutset",
    "sgufp_loopback_create", "sgufp_loopback_destroy", "sgufp_comm_init_loopback",
    "sgufp_subproblem_warm", "sgufp_subproblem_stats",
]


class BnbStats(C.Structure):
    """sgufp_bnb_stats (include/sgufp_hip.h)."""
    _fields_ = [(f, C.c_int64) for f in (
        "popped", "relaxed", "pruned_bound", "pruned_feasibility", "pruned_optimality", "exact", "exact_closed",
        "subproblems", "new_feasibility_cuts", "new_optimality_cuts", "children", "pushed", "frontier",
        "dd_nodes", "dd_arcs", "sweeps")] + [("refine_iters", C.c_int32), ("improved", C.c_int32),
                                             ("ms_relax", C.c_double), ("deferred", C.c_int64),
                                             ("resumed", C.c_int64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class NetworkInfo(C.Structure):
    _fields_ = [("n", C.c_int32), ("m", C.c_int32), ("scenarios", C.c_int32), ("total_layers", C.c_int32),
                ("n_vbar", C.c_int32), ("max_states", C.c_int32), ("n_slots", C.c_int32),
                ("max_batch", C.c_int32), ("node_capacity", C.c_int64), ("arc_capacity", C.c_int64),
                ("scratch_bytes", C.c_int64)]


_lib = None


def comm_unique_id() -> bytes:
    """sgufp_comm_unique_id: the RCCL communicator id, made on one rank."""
    lib = load_library()
    buf = (C.c_uint8 * 128)()
    if lib.sgufp_comm_unique_id(buf, 128) != 0:
        raise RuntimeError("sgufp_comm_unique_id failed")
    return bytes(buf)


def balance_plan(sizes):
    """sgufp_balance_plan (host only): (give[world], idle ranks, chunk_lo / chunk_hi [world,
    world]) of the work sharing sgufp_frontier_balance does for these stack sizes."""
    lib = load_library()
    w = len(sizes)
    sz = np.asarray(sizes, dtype=np.int64)
    give = np.zeros(w, dtype=np.int64)
    idle = np.zeros(w, dtype=np.int32)
    lo = np.zeros((w, w), dtype=np.int64)
    hi = np.zeros((w, w), dtype=np.int64)
    ni = lib.sgufp_balance_plan(w, _ptr(sz), _ptr(give), _ptr(idle), _ptr(lo), _ptr(hi))
    if ni < 0:
        raise ValueError("sgufp_balance_plan: bad sizes")
    return give, [int(x) for x in idle[:ni]], lo[:, :ni], hi[:, :ni]


def load_library(path: str = LIB_PATH) -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    lib = C.CDLL(path)
    P = C.c_void_p
    lib.sgufp_create_from_file.restype = P
    lib.sgufp_create_from_file.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int)]
    lib.sgufp_create.restype = P
    lib.sgufp_destroy.argtypes = [P]
    lib.sgufp_get_network_info.argtypes = [P, C.POINTER(NetworkInfo)]
    lib.sgufp_processing_order.argtypes = [P, P, P]
    lib.sgufp_last_error.restype = C.c_char_p
    lib.sgufp_last_error.argtypes = [P]
    lib.sgufp_stream.restype = P
    lib.sgufp_stream.argtypes = [P]
    lib.sgufp_cuts_append.argtypes = [P, C.c_int, C.c_int, P, P, P, P]
    lib.sgufp_cuts_clear.argtypes = [P]
    lib.sgufp_cuts_count.argtypes = [P, C.c_int]
    lib.sgufp_batch_upload.argtypes = [P, C.c_int, P, P, P, P, P, P, P]
    lib.sgufp_batch_relax.argtypes = [P, C.c_double]
    lib.sgufp_batch_sync.argtypes = [P]
    lib.sgufp_batch_results.argtypes = [P, P, P, P, P, P]
    lib.sgufp_batch_children_size.argtypes = [P, P, P, P]
    lib.sgufp_batch_children.argtypes = [P, P, P, P, P, P, P, P, P]
    lib.sgufp_batch_paths.argtypes = [P, P, P]
    lib.sgufp_batch_stats.argtypes = [P, P, P, P, P]
    lib.sgufp_batch_refine.argtypes = [P, C.c_int, P, P, P, C.c_double]
    lib.sgufp_set_timing.argtypes = [P, C.c_int]
    lib.sgufp_last_timing.argtypes = [P, P, P]
    lib.sgufp_probe_network.argtypes = [C.c_char_p, P, P, C.c_int32, P, P]
    lib.sgufp_batch_debug.argtypes = [P, P, P]
    lib.sgufp_batch_phases.argtypes = [P, P]
    lib.sgufp_batch_routes.argtypes = [P, P]
    lib.sgufp_subproblem.argtypes = [P, C.c_int, P, P, P, P, P, P]
    lib.sgufp_subproblem_detail.argtypes = [P, P, P, P]
    lib.sgufp_slot_keys.argtypes = [P, P]
    lib.sgufp_cuts_append_rows.argtypes = [P, C.c_int, C.c_int, P, P]
    lib.sgufp_frontier_clear.argtypes = [P]
    lib.sgufp_frontier_size.argtypes = [P, P, P]
    lib.sgufp_frontier_push.argtypes = [P, C.c_int, P, P, P, P, P, P, P]
    lib.sgufp_frontier_take_size.argtypes = [P, C.c_int, C.c_int, P, P]
    lib.sgufp_frontier_take.argtypes = [P, C.c_int, C.c_int, P, P, P, P, P, P, P]
    lib.sgufp_bnb_step.argtypes = [P, C.c_int, P, P]
    lib.sgufp_balance_plan.argtypes = [C.c_int, P, P, P, P, P]
    lib.sgufp_comm_allgather_i64.argtypes = [P, P, C.c_int, P]
    lib.sgufp_frontier_peek_size.argtypes = [P, C.c_int64, C.c_int, P, P]
    lib.sgufp_frontier_peek.argtypes = [P, C.c_int64, C.c_int, P, P, P, P, P, P, P]
    lib.sgufp_bnb_set_limits.argtypes = [P, C.c_int, C.c_double]
    lib.sgufp_bnb_set_trace.argtypes = [P, C.c_int]
    lib.sgufp_bnb_trace.argtypes = [P, C.c_int, P, P, P, P, P, P, P, P]
    lib.sgufp_comm_unique_id.argtypes = [P, C.c_int]
    lib.sgufp_comm_init.argtypes = [P, C.c_int, C.c_int, P]
    lib.sgufp_comm_info.argtypes = [P, P, P]
    lib.sgufp_comm_destroy.argtypes = [P]
    lib.sgufp_comm_destroy.restype = None
    lib.sgufp_incumbent_allreduce.argtypes = [P, P]
    lib.sgufp_cuts_exchange.argtypes = [P, P]
    lib.sgufp_frontier_sizes.argtypes = [P, P]
    lib.sgufp_frontier_balance.argtypes = [P, P]
    lib.sgufp_cuts_rows.argtypes = [P, C.c_int, C.c_int, C.c_int, P, P]
    lib.sgufp_restricted_relax.argtypes = [P, C.c_int, C.c_double]
    lib.sgufp_restricted_results.argtypes = [P, P, P, P, P, P]
    lib.sgufp_restricted_paths.argtypes = [P, P, P]
    lib.sgufp_restricted_cutset_size.argtypes = [P, P, P, P]
    lib.sgufp_restricted_cutset.argtypes = [P, P, P, P, P, P, P, P, P]
    lib.sgufp_subproblem_warm.argtypes = [P, C.c_int, P, P, P, P, P, P, P, P]
    lib.sgufp_subproblem_stats.argtypes = [P, P, P]
    lib.sgufp_loopback_create.restype = P
    lib.sgufp_loopback_create.argtypes = [C.c_int]
    lib.sgufp_loopback_destroy.restype = None
    lib.sgufp_loopback_destroy.argtypes = [P]
    lib.sgufp_comm_init_loopback.argtypes = [P, P, C.c_int]
    lib.sgufp_dd_build.argtypes = [P]
    lib.sgufp_dd_apply.argtypes = [P, C.c_int, C.c_int, C.c_double, C.c_int64, P, P, C.c_double, P]
    lib.sgufp_dd_solution.argtypes = [P, C.c_int, P, P]
    lib.sgufp_dd_cutset.argtypes = [P, C.c_int, C.c_double, P]
    _lib = lib
    return lib


class LoopbackGroup:
    """sgufp_loopback_create(world): `world` contexts of this process exchanging through the
    library's shard protocol with device-to-device copies (Engine.comm_init_loopback)."""

    def __init__(self, world: int):
        self.lib = load_library()
        self.world = world
        self.handle = self.lib.sgufp_loopback_create(int(world))
        if not self.handle:
            raise RuntimeError("sgufp_loopback_create failed")

    def close(self):
        if self.handle:
            self.lib.sgufp_loopback_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def key_of(q: int, i: int, j: int) -> int:
    """Inavap::getKey (Cut.h:342-344)."""
    return (q & 0xFFFF) | ((i & 0xFFFF) << 16) | ((j & 0xFFFF) << 32)


def pack_cuts(cuts: Sequence[PoolCut]):
    """cutToCut (Cut.h:406-421): (i,q,j) map order, zero coefficients dropped."""
    rhs = np.array([c.rhs for c in cuts], dtype=np.float64)
    off = [0]
    keys: List[int] = []
    vals: List[float] = []
    for c in cuts:
        for (i, q, j, v) in sorted(c.coeff, key=lambda t: (t[0], t[1], t[2])):
            if v == 0.0:
                continue
            keys.append(key_of(q, i, j))
            vals.append(v)
        off.append(len(keys))
    return rhs, np.array(off, dtype=np.int64), np.array(keys, dtype=np.uint64), np.array(vals, dtype=np.float64)


def probe_network(path: str):
    """Host-only parse through the product loader: (totalLayers, processingOrder arcs, V-bar order)."""
    lib = load_library()
    L, nv = C.c_int32(0), C.c_int32(0)
    if lib.sgufp_probe_network(path.encode(), C.byref(L), C.byref(nv), 0, None, None) != 0:
        raise RuntimeError(f"cannot parse {path}")
    cap = max(L.value, nv.value, 1)
    la = np.zeros(cap, dtype=np.int32)
    vb = np.zeros(cap, dtype=np.int32)
    lib.sgufp_probe_network(path.encode(), C.byref(L), C.byref(nv), cap, _ptr(la), _ptr(vb))
    return L.value, la[:L.value].copy(), vb[:nv.value].copy()


class BatchArrays:
    """SoA view of a list of Inavap::Node records."""

    def __init__(self, nodes: Sequence[NodeRecord]):
        n = len(nodes)
        self.n = n
        self.gl = np.array([nd.gl for nd in nodes], dtype=np.uint16)
        self.lb = np.array([nd.lb for nd in nodes], dtype=np.float64)
        self.ub = np.array([nd.ub for nd in nodes], dtype=np.float64)
        st_len = np.array([len(nd.states) for nd in nodes], dtype=np.int64)
        so_len = np.array([len(nd.sol) for nd in nodes], dtype=np.int64)
        self.states_off = np.zeros(n + 1, dtype=np.int64)
        self.sol_off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(st_len, out=self.states_off[1:])
        np.cumsum(so_len, out=self.sol_off[1:])
        self.states = np.array([s for nd in nodes for s in nd.states], dtype=np.int16)
        self.sol = np.array([s for nd in nodes for s in nd.sol], dtype=np.int16)


def batch_from_arrays(gl, lb, ub, states_off, states, sol_off, sol) -> BatchArrays:
    b = BatchArrays.__new__(BatchArrays)
    b.n = int(len(gl))
    b.gl = np.ascontiguousarray(gl, dtype=np.uint16)
    b.lb = np.ascontiguousarray(lb, dtype=np.float64)
    b.ub = np.ascontiguousarray(ub, dtype=np.float64)
    b.states_off = np.ascontiguousarray(states_off, dtype=np.int64)
    b.states = np.ascontiguousarray(states, dtype=np.int16)
    b.sol_off = np.ascontiguousarray(sol_off, dtype=np.int64)
    b.sol = np.ascontiguousarray(sol, dtype=np.int16)
    return b


def batch_slice(b: BatchArrays, idx: np.ndarray) -> BatchArrays:
    """Sub-batch of the records at positions ``idx`` (in that order)."""
    idx = np.asarray(idx, dtype=np.int64)
    st_len = b.states_off[idx + 1] - b.states_off[idx]
    so_len = b.sol_off[idx + 1] - b.sol_off[idx]
    st_off = np.zeros(len(idx) + 1, dtype=np.int64)
    so_off = np.zeros(len(idx) + 1, dtype=np.int64)
    np.cumsum(st_len, out=st_off[1:])
    np.cumsum(so_len, out=so_off[1:])
    st = np.concatenate([b.states[b.states_off[k]:b.states_off[k + 1]] for k in idx]) if len(idx) else b.states[:0]
    so = np.concatenate([b.sol[b.sol_off[k]:b.sol_off[k + 1]] for k in idx]) if len(idx) else b.sol[:0]
    return batch_from_arrays(b.gl[idx], b.lb[idx], b.ub[idx], st_off, st, so_off, so)


def batch_concat(parts: Sequence[BatchArrays]) -> BatchArrays:
    gl = np.concatenate([p.gl for p in parts])
    lb = np.concatenate([p.lb for p in parts])
    ub = np.concatenate([p.ub for p in parts])
    st = np.concatenate([p.states for p in parts])
    so = np.concatenate([p.sol for p in parts])
    st_off = [np.zeros(1, dtype=np.int64)]
    so_off = [np.zeros(1, dtype=np.int64)]
    a = b_ = 0
    for p in parts:
        st_off.append(p.states_off[1:] + a)
        so_off.append(p.sol_off[1:] + b_)
        a += int(p.states_off[-1])
        b_ += int(p.sol_off[-1])
    return batch_from_arrays(gl, lb, ub, np.concatenate(st_off), st, np.concatenate(so_off), so)


def batch_to_records(b: BatchArrays) -> List[NodeRecord]:
    return [NodeRecord(int(b.gl[k]), float(b.lb[k]), float(b.ub[k]),
                       [int(x) for x in b.states[b.states_off[k]:b.states_off[k + 1]]],
                       [int(x) for x in b.sol[b.sol_off[k]:b.sol_off[k + 1]]]) for k in range(b.n)]


class Engine:
    """One device context: network tables, cut pools, a batch of DD slots."""

    def __init__(self, network_path: str, device: int = 0, max_batch: int = 4096):
        self.lib = load_library()
        self.device = device
        err = C.c_int(0)
        self.ctx = self.lib.sgufp_create_from_file(network_path.encode(), device, max_batch, C.byref(err))
        if not self.ctx:
            raise RuntimeError(f"sgufp_create_from_file failed ({err.value})")
        self.info = NetworkInfo()
        self._check(self.lib.sgufp_get_network_info(self.ctx, C.byref(self.info)))
        self.n_feas = 0
        self.n_opt = 0
        self.n = 0

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.sgufp_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != 0:
            raise RuntimeError(f"sgufp call failed ({rc}): {self.lib.sgufp_last_error(self.ctx).decode()}")

    # -- network -------------------------------------------------------------
    def processing_order(self) -> Tuple[np.ndarray, np.ndarray]:
        la = np.zeros(self.info.total_layers, dtype=np.int32)
        vb = np.zeros(self.info.n_vbar, dtype=np.int32)
        self._check(self.lib.sgufp_processing_order(self.ctx, _ptr(la), _ptr(vb)))
        return la, vb

    # -- cuts ----------------------------------------------------------------
    def add_cuts(self, cuts: Sequence[PoolCut]):
        """Append in insertion order, split by type (two Containers, DDSolver.h:415-416)."""
        for t in (1, 0):
            sel = [c for c in cuts if c.type == t]
            if not sel:
                continue
            rhs, off, keys, vals = pack_cuts(sel)
            self._check(self.lib.sgufp_cuts_append(self.ctx, t, len(sel), _ptr(rhs), _ptr(off), _ptr(keys), _ptr(vals)))
            if t == 1:
                self.n_feas += len(sel)
            else:
                self.n_opt += len(sel)

    def clear_cuts(self):
        self._check(self.lib.sgufp_cuts_clear(self.ctx))
        self.n_feas = self.n_opt = 0

    # -- batch ---------------------------------------------------------------
    def upload(self, nodes: Sequence[NodeRecord] | BatchArrays):
        b = nodes if isinstance(nodes, BatchArrays) else BatchArrays(nodes)
        self._check(self.lib.sgufp_batch_upload(self.ctx, b.n, _ptr(b.gl), _ptr(b.lb), _ptr(b.ub), _ptr(b.states_off),
                                                _ptr(b.states), _ptr(b.sol_off), _ptr(b.sol)))
        self.n = b.n

    def relax_async(self, incumbent: float):
        self._check(self.lib.sgufp_batch_relax(self.ctx, C.c_double(incumbent)))

    def sync(self):
        self._check(self.lib.sgufp_batch_sync(self.ctx))

    def set_timing(self, on: bool):
        self._check(self.lib.sgufp_set_timing(self.ctx, 1 if on else 0))

    def last_timing(self) -> Tuple[float, float]:
        a, b = C.c_float(0), C.c_float(0)
        self._check(self.lib.sgufp_last_timing(self.ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def results_arrays(self):
        n = self.n
        st = np.zeros(n, dtype=np.int32)
        ex = np.zeros(n, dtype=np.uint8)
        lb = np.zeros(n, dtype=np.float64)
        ub = np.zeros(n, dtype=np.float64)
        nc = np.zeros(n, dtype=np.int32)
        self._check(self.lib.sgufp_batch_results(self.ctx, _ptr(st), _ptr(ex), _ptr(lb), _ptr(ub), _ptr(nc)))
        return st, ex, lb, ub, nc

    def stats(self):
        n = self.n
        a = np.zeros(n, dtype=np.int64)
        b = np.zeros(n, dtype=np.int64)
        c = np.zeros(n, dtype=np.int32)
        d = np.zeros(n, dtype=np.int32)
        self._check(self.lib.sgufp_batch_stats(self.ctx, _ptr(a), _ptr(b), _ptr(c), _ptr(d)))
        return a, b, c, d

    def children_arrays(self):
        n = self.n
        nc, ns, nsol = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        self._check(self.lib.sgufp_batch_children_size(self.ctx, C.byref(nc), C.byref(ns), C.byref(nsol)))
        k = nc.value
        child_off = np.zeros(n + 1, dtype=np.int64)
        gl = np.zeros(k, dtype=np.uint16)
        lb = np.zeros(k, dtype=np.float64)
        ub = np.zeros(k, dtype=np.float64)
        soff = np.zeros(k + 1, dtype=np.int64)
        states = np.zeros(max(ns.value, 1), dtype=np.int16)
        poff = np.zeros(k + 1, dtype=np.int64)
        sol = np.zeros(max(nsol.value, 1), dtype=np.int16)
        self._check(self.lib.sgufp_batch_children(self.ctx, _ptr(child_off), _ptr(gl), _ptr(lb), _ptr(ub), _ptr(soff),
                                                  _ptr(states), _ptr(poff), _ptr(sol)))
        return child_off, gl, lb, ub, soff, states, poff, sol

    def debug(self):
        t = np.zeros(self.n, dtype=np.int64)
        r = np.zeros(self.n, dtype=np.int32)
        self._check(self.lib.sgufp_batch_debug(self.ctx, _ptr(t), _ptr(r)))
        return t, r

    def phases(self):
        t = np.zeros((self.n, 8), dtype=np.int64)
        self._check(self.lib.sgufp_batch_phases(self.ctx, _ptr(t)))
        return t

    def children_batch(self) -> BatchArrays:
        """All cutset children of the last relaxed batch as a new batch (node order kept)."""
        child_off, gl, lb, ub, soff, states, poff, sol = self.children_arrays()
        return batch_from_arrays(gl, lb, ub, soff, states[:soff[-1]], poff, sol[:poff[-1]])

    def paths(self):
        n = self.n
        off = np.zeros(n + 1, dtype=np.int64)
        self._check(self.lib.sgufp_batch_paths(self.ctx, _ptr(off), None))
        buf = np.zeros(max(int(off[-1]), 1), dtype=np.int16)
        self._check(self.lib.sgufp_batch_paths(self.ctx, _ptr(off), _ptr(buf)))
        return off, buf

    def refine(self, node_idx: Sequence[int], is_feas: Sequence[int], cut_index: Sequence[int], incumbent: float):
        ni = np.asarray(node_idx, dtype=np.int32)
        fe = np.asarray(is_feas, dtype=np.uint8)
        ci = np.asarray(cut_index, dtype=np.int32)
        self._check(self.lib.sgufp_batch_refine(self.ctx, len(ni), _ptr(ni), _ptr(fe), _ptr(ci), C.c_double(incumbent)))

    def routes(self) -> np.ndarray:
        """Per staged record, which kernels took its optimality phase in the last relaxation
        (sgufp_batch_routes): ROUTE_IN_ORDER, ROUTE_EXACT_PHASE, ROUTE_NX_PHASE, ROUTE_NX_FALLBACK."""
        r = np.zeros(max(self.n, 1), dtype=np.int32)
        self._check(self.lib.sgufp_batch_routes(self.ctx, _ptr(r)))
        return r[:self.n]

    # -- one DD at a time: Inavap::RelaxedDDNew (DD.h:797-808) ----------------
    def dd_build(self, nodes):
        """buildTree for each record, no cut applied; returns the exact flags (isTreeExact)."""
        self.upload(nodes)
        self._check(self.lib.sgufp_dd_build(self.ctx))
        _st, ex, _lb, _ub, _nc = self.results_arrays()
        return ex

    def dd_apply(self, node: int, cut: PoolCut, optimal: float) -> float:
        """applyFeasibilityCut (1.0 / 0.0) or applyOptimalityCut (the returned bound) of one cut."""
        keys = np.asarray([key_of(q, i, j) for (i, q, j, _v) in cut.coeff], dtype=np.uint64)
        vals = np.asarray([v for (_i, _q, _j, v) in cut.coeff], dtype=np.float64)
        out = np.zeros(1, dtype=np.float64)
        self._check(self.lib.sgufp_dd_apply(self.ctx, int(node), int(cut.type), C.c_double(cut.rhs), len(keys),
                                            _ptr(keys), _ptr(vals), C.c_double(optimal), _ptr(out)))
        return float(out[0])

    def dd_solution(self, node: int) -> List[int]:
        buf = np.zeros(max(self.info.total_layers, 1), dtype=np.int16)
        n = C.c_int32(0)
        self._check(self.lib.sgufp_dd_solution(self.ctx, int(node), _ptr(buf), C.byref(n)))
        return [int(x) for x in buf[:n.value]]

    def dd_cutset(self, node: int, ub: float) -> List[NodeRecord]:
        nc = C.c_int64(0)
        self._check(self.lib.sgufp_dd_cutset(self.ctx, int(node), C.c_double(ub), C.byref(nc)))
        child_off, gl, clb, cub, soff, states, poff, sol = self.children_arrays()
        return [NodeRecord(int(gl[c]), float(clb[c]), float(cub[c]), [int(x) for x in states[soff[c]:soff[c + 1]]],
                           [int(x) for x in sol[poff[c]:poff[c + 1]]]) for c in range(int(nc.value))]

    # -- scenario subproblem ---------------------------------------------------
    def slot_keys(self) -> np.ndarray:
        keys = np.zeros(max(self.info.n_slots, 1), dtype=np.uint64)
        self._check(self.lib.sgufp_slot_keys(self.ctx, _ptr(keys)))
        return keys[:self.info.n_slots]

    def restricted(self, nodes, incumbent: float, width: int = 128):
        """Inavap::RestrictedDDNew{net, width} for each record under the pool (restricted
        cut phases of NodeExplorer::processX3, NodeExplorer.cpp:605-656), on the device.
        Returns per record (status, exact, lb, max path, exact cutset records)."""
        self.upload(nodes)
        self._check(self.lib.sgufp_restricted_relax(self.ctx, int(width), C.c_double(incumbent)))
        n = len(nodes) if not isinstance(nodes, BatchArrays) else nodes.n
        st = np.zeros(max(n, 1), dtype=np.int32)
        ex = np.zeros(max(n, 1), dtype=np.uint8)
        lb = np.zeros(max(n, 1), dtype=np.float64)
        pl = np.zeros(max(n, 1), dtype=np.int32)
        cn = np.zeros(max(n, 1), dtype=np.int32)
        self._check(self.lib.sgufp_restricted_results(self.ctx, _ptr(st), _ptr(ex), _ptr(lb), _ptr(pl), _ptr(cn)))
        off = np.zeros(n + 1, dtype=np.int64)
        self._check(self.lib.sgufp_restricted_paths(self.ctx, _ptr(off), None))
        buf = np.zeros(max(int(off[n]), 1), dtype=np.int16)
        self._check(self.lib.sgufp_restricted_paths(self.ctx, _ptr(off), _ptr(buf)))
        nr, ns, nsol = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        self._check(self.lib.sgufp_restricted_cutset_size(self.ctx, C.byref(nr), C.byref(ns), C.byref(nsol)))
        R = nr.value
        roff = np.zeros(n + 1, dtype=np.int64)
        gl = np.zeros(max(R, 1), dtype=np.uint16)
        clb = np.zeros(max(R, 1), dtype=np.float64)
        cub = np.zeros(max(R, 1), dtype=np.float64)
        soff = np.zeros(R + 1, dtype=np.int64)
        states = np.zeros(max(ns.value, 1), dtype=np.int16)
        poff = np.zeros(R + 1, dtype=np.int64)
        sol = np.zeros(max(nsol.value, 1), dtype=np.int16)
        self._check(self.lib.sgufp_restricted_cutset(self.ctx, _ptr(roff), _ptr(gl), _ptr(clb), _ptr(cub), _ptr(soff),
                                                     _ptr(states), _ptr(poff), _ptr(sol)))
        out = []
        for k in range(n):
            kids = []
            for r in range(int(roff[k]), int(roff[k + 1])):
                kids.append(NodeRecord(int(gl[r]), float(clb[r]), float(cub[r]),
                                       [int(x) for x in states[soff[r]:soff[r + 1]]],
                                       [int(x) for x in sol[poff[r]:poff[r + 1]]]))
            out.append((int(st[k]), int(ex[k]), float(lb[k]), [int(x) for x in buf[off[k]:off[k + 1]]], kids))
        return out

    def subproblem(self, paths: Sequence[Sequence[int]], warm_src: Optional[Sequence[int]] = None,
                   warm_dst: Optional[Sequence[int]] = None):
        """GuroSolver::solveSubProblem for each path on the device; with warm_src / warm_dst,
        path k starts from ring slot warm_src[k] and stores its state in warm_dst[k]
        (sgufp_subproblem_warm).

        Returns (type[n], rhs[n], rows[n, n_slots + 1], obj_mean[n]); type 0 optimality,
        1 feasibility, -1 error."""
        n = len(paths)
        off = np.zeros(n + 1, dtype=np.int64)
        for k, p in enumerate(paths):
            off[k + 1] = off[k] + len(p)
        flat = np.concatenate([np.asarray(p, dtype=np.int16) for p in paths]) if n else np.zeros(1, np.int16)
        if flat.size == 0:
            flat = np.zeros(1, np.int16)
        typ = np.zeros(max(n, 1), dtype=np.int32)
        rhs = np.zeros(max(n, 1), dtype=np.float64)
        rows = np.zeros((max(n, 1), self.info.n_slots + 1), dtype=np.float64)
        obj = np.zeros(max(n, 1), dtype=np.float64)
        if warm_src is None:
            self._check(self.lib.sgufp_subproblem(self.ctx, n, _ptr(off), _ptr(flat), _ptr(typ), _ptr(rhs),
                                                  _ptr(rows), _ptr(obj)))
        else:
            src = np.asarray(warm_src, dtype=np.int32)
            dst = np.asarray(warm_dst, dtype=np.int32)
            self._check(self.lib.sgufp_subproblem_warm(self.ctx, n, _ptr(off), _ptr(flat), _ptr(src), _ptr(dst),
                                                       _ptr(typ), _ptr(rhs), _ptr(rows), _ptr(obj)))
        return typ[:n], rhs[:n], rows[:n], obj[:n]

    def subproblem_stats(self, n: int):
        """Per (path, scenario) of the last call: augmenting paths (negative: a warm start fell
        back cold) and Bellman-Ford passes, each [n, S]."""
        S = self.info.scenarios
        a = np.zeros(max(n * S, 1), dtype=np.int32)
        p = np.zeros(max(n * S, 1), dtype=np.int32)
        self._check(self.lib.sgufp_subproblem_stats(self.ctx, _ptr(a), _ptr(p)))
        return a[:n * S].reshape(n, S), p[:n * S].reshape(n, S)

    def subproblem_detail(self, n: int):
        """Per (path, scenario) status / primal objective / dual objective of the last call."""
        S = self.info.scenarios
        st = np.zeros(max(n * S, 1), dtype=np.int32)
        ob = np.zeros(max(n * S, 1), dtype=np.float64)
        du = np.zeros(max(n * S, 1), dtype=np.float64)
        self._check(self.lib.sgufp_subproblem_detail(self.ctx, _ptr(st), _ptr(ob), _ptr(du)))
        return st[:n * S].reshape(n, S), ob[:n * S].reshape(n, S), du[:n * S].reshape(n, S)

    def add_cut_rows(self, is_feas: int, rhs: np.ndarray, rows: np.ndarray):
        rhs = np.ascontiguousarray(rhs, dtype=np.float64)
        rows = np.ascontiguousarray(rows, dtype=np.float64)
        self._check(self.lib.sgufp_cuts_append_rows(self.ctx, int(is_feas), len(rhs), _ptr(rhs), _ptr(rows)))

    def cut_rows(self, is_feas: int, first: int = 0, count: Optional[int] = None):
        """Pool cuts of one list (insertion order) as (rhs[k], rows[k, n_slots + 1])."""
        total = self.lib.sgufp_cuts_count(self.ctx, int(is_feas))
        count = total - first if count is None else count
        rhs = np.zeros(max(count, 1), dtype=np.float64)
        rows = np.zeros((max(count, 1), self.info.n_slots + 1), dtype=np.float64)
        self._check(self.lib.sgufp_cuts_rows(self.ctx, int(is_feas), first, count, _ptr(rhs), _ptr(rows)))
        return rhs[:count], rows[:count]

    def cuts_count(self, is_feas: int) -> int:
        return int(self.lib.sgufp_cuts_count(self.ctx, int(is_feas)))

    # -- device frontier + B&B rounds (Inavap::DDSolver) -------------------------
    def frontier_clear(self):
        self._check(self.lib.sgufp_frontier_clear(self.ctx))

    def frontier_size(self) -> int:
        n = C.c_int64(0)
        self._check(self.lib.sgufp_frontier_size(self.ctx, C.byref(n), None))
        return n.value

    def frontier_push(self, nodes: Sequence[NodeRecord] | BatchArrays):
        b = nodes if isinstance(nodes, BatchArrays) else BatchArrays(nodes)
        self._check(self.lib.sgufp_frontier_push(self.ctx, b.n, _ptr(b.gl), _ptr(b.lb), _ptr(b.ub), _ptr(b.states_off),
                                                 _ptr(b.states), _ptr(b.sol_off), _ptr(b.sol)))

    def frontier_take(self, n: int, from_bottom: bool = True) -> BatchArrays:
        ns, nl = C.c_int64(0), C.c_int64(0)
        fb = 1 if from_bottom else 0
        self._check(self.lib.sgufp_frontier_take_size(self.ctx, n, fb, C.byref(ns), C.byref(nl)))
        gl = np.zeros(max(n, 1), dtype=np.uint16)
        lb = np.zeros(max(n, 1), dtype=np.float64)
        ub = np.zeros(max(n, 1), dtype=np.float64)
        soff = np.zeros(n + 1, dtype=np.int64)
        states = np.zeros(max(ns.value, 1), dtype=np.int16)
        poff = np.zeros(n + 1, dtype=np.int64)
        sol = np.zeros(max(nl.value, 1), dtype=np.int16)
        self._check(self.lib.sgufp_frontier_take(self.ctx, n, fb, _ptr(gl), _ptr(lb), _ptr(ub), _ptr(soff),
                                                 _ptr(states), _ptr(poff), _ptr(sol)))
        return batch_from_arrays(gl[:n], lb[:n], ub[:n], soff, states[:ns.value], poff, sol[:nl.value])

    def frontier_peek(self, first: int, n: int) -> BatchArrays:
        """Copies of the records at stack positions [first, first + n) (0 = bottom), left in place."""
        ns, nl = C.c_int64(0), C.c_int64(0)
        self._check(self.lib.sgufp_frontier_peek_size(self.ctx, int(first), n, C.byref(ns), C.byref(nl)))
        gl = np.zeros(max(n, 1), dtype=np.uint16)
        lb = np.zeros(max(n, 1), dtype=np.float64)
        ub = np.zeros(max(n, 1), dtype=np.float64)
        soff = np.zeros(n + 1, dtype=np.int64)
        states = np.zeros(max(ns.value, 1), dtype=np.int16)
        poff = np.zeros(n + 1, dtype=np.int64)
        sol = np.zeros(max(nl.value, 1), dtype=np.int16)
        self._check(self.lib.sgufp_frontier_peek(self.ctx, int(first), n, _ptr(gl), _ptr(lb), _ptr(ub), _ptr(soff),
                                                 _ptr(states), _ptr(poff), _ptr(sol)))
        return batch_from_arrays(gl[:n], lb[:n], ub[:n], soff, states[:ns.value], poff, sol[:nl.value])

    def bnb_step(self, incumbent: float, max_nodes: int = 0) -> Tuple[float, BnbStats]:
        """One batched B&B round; returns the new incumbent and the round's counters."""
        z = C.c_double(incumbent)
        st = BnbStats()
        self._check(self.lib.sgufp_bnb_step(self.ctx, int(max_nodes), C.byref(z), C.byref(st)))
        return z.value, st

    def bnb_set_limits(self, max_refine_iters: int = 0, round_seconds: float = 0.0):
        """Bound the refinement loops of one bnb_step (0: no limit); unfinished exact
        records go back on top of the frontier."""
        self._check(self.lib.sgufp_bnb_set_limits(self.ctx, int(max_refine_iters), C.c_double(round_seconds)))

    def bnb_set_trace(self, on: bool = True):
        """Keep what each bnb_step round did (sgufp_bnb_set_trace) for bnb_trace()."""
        self._check(self.lib.sgufp_bnb_set_trace(self.ctx, 1 if on else 0))

    def bnb_trace(self, kind: int):
        """The last round's trace of one kind (0 popped records, 1 subproblems, 2 closed
        loops; include/sgufp_hip.h): a list of (record, code, row, value, path)."""
        n, pe = C.c_int64(0), C.c_int64(0)
        self._check(self.lib.sgufp_bnb_trace(self.ctx, int(kind), C.byref(n), C.byref(pe), None, None, None, None,
                                             None, None))
        k = n.value
        rec = np.zeros(max(k, 1), dtype=np.int32)
        code = np.zeros(max(k, 1), dtype=np.int32)
        row = np.zeros(max(k, 1), dtype=np.int32)
        val = np.zeros(max(k, 1), dtype=np.float64)
        off = np.zeros(k + 1, dtype=np.int64)
        paths = np.zeros(max(pe.value, 1), dtype=np.int16)
        self._check(self.lib.sgufp_bnb_trace(self.ctx, int(kind), C.byref(n), C.byref(pe), _ptr(rec), _ptr(code),
                                             _ptr(row), _ptr(val), _ptr(off), _ptr(paths)))
        return [(int(rec[i]), int(code[i]), int(row[i]), float(val[i]), [int(x) for x in paths[off[i]:off[i + 1]]])
                for i in range(k)]

    # -- frontier shards over RCCL (shard.cpp) --------------------------------------
    def comm_init(self, world: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.sgufp_comm_init(self.ctx, int(world), int(rank), buf))

    def comm_init_loopback(self, group: "LoopbackGroup", rank: int):
        """This context as shard `rank` of an in-process loopback group (shard.cpp): the
        library's own exchanges between contexts of this process, one host thread each."""
        self._check(self.lib.sgufp_comm_init_loopback(self.ctx, group.handle, int(rank)))

    def incumbent_allreduce(self, z: float) -> float:
        v = C.c_double(z)
        self._check(self.lib.sgufp_incumbent_allreduce(self.ctx, C.byref(v)))
        return v.value

    def cuts_exchange(self) -> int:
        n = C.c_int64(0)
        self._check(self.lib.sgufp_cuts_exchange(self.ctx, C.byref(n)))
        return n.value

    def frontier_sizes(self, world: int) -> List[int]:
        a = (C.c_int64 * max(world, 1))()
        self._check(self.lib.sgufp_frontier_sizes(self.ctx, a))
        return [int(x) for x in a]

    def comm_allgather_i64(self, vals: Sequence[int], world: int) -> np.ndarray:
        """[world, len(vals)] (len <= 4) over the context's communicator (sgufp_comm_allgather_i64)."""
        v = np.asarray(list(vals), dtype=np.int64)
        out = np.zeros(max(world * len(v), 1), dtype=np.int64)
        self._check(self.lib.sgufp_comm_allgather_i64(self.ctx, _ptr(v), len(v), _ptr(out)))
        return out[:world * len(v)].reshape(world, len(v))

    def frontier_balance(self) -> int:
        n = C.c_int64(0)
        self._check(self.lib.sgufp_frontier_balance(self.ctx, C.byref(n)))
        return n.value

    # -- convenience: NodeExplorer::process for a list of nodes ----------------
    def relax(self, nodes: Sequence[NodeRecord], incumbent: float) -> List[RelaxResult]:
        out: List[RelaxResult] = []
        for s in range(0, len(nodes), self.info.max_batch):
            chunk = nodes[s:s + self.info.max_batch]
            self.upload(chunk)
            self.relax_async(incumbent)
            self.sync()
            out.extend(self._collect())
        return out

    def _collect(self) -> List[RelaxResult]:
        st, ex, lb, ub, nc = self.results_arrays()
        dn, da, dl, _ = self.stats()
        child_off, gl, clb, cub, soff, states, poff, sol = self.children_arrays()
        p_off, pbuf = self.paths()
        res = []
        for k in range(self.n):
            ch = []
            for c in range(int(child_off[k]), int(child_off[k + 1])):
                ch.append(NodeRecord(int(gl[c]), float(clb[c]), float(cub[c]),
                                     [int(x) for x in states[soff[c]:soff[c + 1]]],
                                     [int(x) for x in sol[poff[c]:poff[c + 1]]]))
            path = [int(x) for x in pbuf[p_off[k]:p_off[k + 1]]]
            res.append(RelaxResult(int(st[k]), int(ex[k]), float(lb[k]), float(ub[k]), ch, path,
                                   int(dn[k]), int(da[k]), int(dl[k])))
        return res
