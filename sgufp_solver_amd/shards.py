"""Exchanges between frontier shards -- one process per GPU, ``torch.distributed`` with the
"nccl" backend (RCCL over xGMI) on the GPUs, "gloo" in the CPU tests.

The reference shares one address space between its master and worker threads
(/root/reference/DDSolver.cpp:556-846); the sharded solver replaces each shared-memory
exchange by a collective on fixed-shape tensors (no pickled objects):

* incumbent: all-reduce(MAX) of one f64 -- the CAS-max on ``DDSolver::optimal``
  (DDSolver.cpp:723-731);
* cut pool: all-gather of the rows each shard appended since the last exchange (counts
  first, then one padded f64 block [k_max, 1 + n_slots + 1] per shard: RHS, dense row) -- the
  global ``feasCutsGlobal`` / ``optCutsGlobal`` Containers every worker reads
  (DDSolver.h:415-416);
* frontier sizes + flags: one all-gather of a few int64 per shard (termination,
  DDSolver.cpp:630-640, and the time budget);
* work sharing: while a shard is idle, every busy shard gives away records from the
  bottom (oldest end) of its stack -- 40 % when it holds at least 32 (``lf_queue::m_pop(0.4)``
  with ``_queue_limit_``, lock_free_queue.h:14,125-164, as the master steals from every
  busy worker, DDSolver.cpp:642-652), half of a smaller stack (the master's ceil(q/2)
  hand-out, DDSolver.cpp:603-621) -- and the idle shards split every donor's records in
  contiguous chunks.  Records travel as one packed byte block per donor.
"""
from __future__ import annotations

import threading
from typing import List, Sequence

import numpy as np

STEAL_SHARE = 0.4    # PROPORTION_OF_SHARE (DDSolver.h:22-38)
QUEUE_LIMIT = 32     # _queue_limit_ (lock_free_queue.h:14): m_pop gives nothing below it


def give_count(size: int) -> int:
    """Records a busy shard of `size` gives to the idle ones."""
    if size >= QUEUE_LIMIT:
        # m_pop: skip int(size * (1 - 0.4)) from the head, hand over the rest from the tail
        return size - int(float(size) * (1.0 - STEAL_SHARE))
    if size >= 2:
        return size // 2
    return 0


def plan(sizes: Sequence[int]):
    """(donors [(rank, count)], idle ranks) -- identical on every rank."""
    idle = [r for r, s in enumerate(sizes) if s == 0]
    if not idle:
        return [], []
    donors = [(r, give_count(int(s))) for r, s in enumerate(sizes) if s > 0]
    donors = [(r, g) for r, g in donors if g > 0]
    return donors, idle


def pack_batch(b) -> np.ndarray:
    """BatchArrays -> one uint8 block (header: n, states, solution entries)."""
    n = int(b.n)
    hdr = np.array([n, int(b.states_off[n]) if n else 0, int(b.sol_off[n]) if n else 0], dtype=np.int64)
    parts = [hdr, np.asarray(b.gl[:n], dtype=np.uint16), np.asarray(b.lb[:n], dtype=np.float64),
             np.asarray(b.ub[:n], dtype=np.float64), np.asarray(b.states_off[:n + 1], dtype=np.int64),
             np.asarray(b.states[:hdr[1]], dtype=np.int16), np.asarray(b.sol_off[:n + 1], dtype=np.int64),
             np.asarray(b.sol[:hdr[2]], dtype=np.int16)]
    return np.concatenate([p.view(np.uint8) for p in parts])


def unpack_batch(buf: np.ndarray):
    from .engine import batch_from_arrays
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    hdr = buf[:24].view(np.int64)
    n, ns, nl = int(hdr[0]), int(hdr[1]), int(hdr[2])
    pos = 24

    def take(dtype, count):
        nonlocal pos
        size = np.dtype(dtype).itemsize * count
        a = buf[pos:pos + size].view(dtype).copy()
        pos += size
        return a
    gl = take(np.uint16, n)
    lb = take(np.float64, n)
    ub = take(np.float64, n)
    so = take(np.int64, n + 1)
    st = take(np.int16, ns)
    po = take(np.int64, n + 1)
    sol = take(np.int16, nl)
    return batch_from_arrays(gl, lb, ub, so, st, po, sol)


class ShardComm:
    """Tensor collectives of one frontier shard over a torch.distributed group."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dev = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(group) == "nccl" else torch.device("cpu")
        self.bytes = 0          # payload bytes this shard put on the wire (all collectives)

    def allreduce_max(self, z: float) -> float:
        t = self.torch.tensor([z], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        self.bytes += 8
        return float(t.item())

    def allgather_i64(self, vals: Sequence[int]) -> np.ndarray:
        """[world, len(vals)] int64."""
        t = self.torch.tensor(list(vals), dtype=self.torch.int64, device=self.dev)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        self.bytes += 8 * len(vals)
        return np.stack([o.cpu().numpy() for o in out])

    def allgather_rows(self, rows: np.ndarray) -> List[np.ndarray]:
        """rows [k, c] f64 (a rank with no rows may pass any c) -> each rank's rows, as one
        padded [k_max, c] block per rank."""
        kc = self.allgather_i64([rows.shape[0], rows.shape[1] if rows.shape[0] else 0])
        k = kc[:, 0]
        c = int(kc[:, 1].max())
        kmax = int(k.max())
        if kmax == 0:
            return [np.zeros((0, c)) for _ in range(self.world)]
        pad = np.zeros((kmax, c), dtype=np.float64)
        if rows.shape[0]:
            pad[:rows.shape[0]] = rows
        t = self.torch.from_numpy(pad).to(self.dev)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        self.bytes += pad.nbytes
        return [out[r][:int(k[r])].cpu().numpy() for r in range(self.world)]

    def allgather_bytes(self, blob: np.ndarray) -> List[np.ndarray]:
        nb = self.allgather_i64([blob.size])[:, 0]
        bmax = int(nb.max())
        if bmax == 0:
            return [np.zeros(0, np.uint8) for _ in range(self.world)]
        pad = np.zeros(bmax, dtype=np.uint8)
        pad[:blob.size] = blob
        t = self.torch.from_numpy(pad).to(self.dev)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        self.bytes += pad.nbytes
        return [out[r][:int(nb[r])].cpu().numpy() for r in range(self.world)]

    # -- the exchanges of one B&B round --------------------------------------------
    def exchange_cuts(self, eng, marks) -> int:
        """All-gather the cut rows appended locally since the last exchange; append the
        other shards' rows in rank order (each list: feasibility, optimality).
        marks[t] = rows of list t already shared; returns rows received."""
        got = 0
        for t in (1, 0):
            n = eng.cuts_count(t)
            if n > marks[t]:
                rhs, rows = eng.cut_rows(t, marks[t], n - marks[t])
                mine = np.concatenate([np.asarray(rhs, dtype=np.float64)[:, None],
                                       np.asarray(rows, dtype=np.float64)], axis=1)
            else:
                mine = np.zeros((0, 0), dtype=np.float64)
            every = self.allgather_rows(mine)
            for r in range(self.world):
                if r == self.rank or every[r].shape[0] == 0:
                    continue
                eng.add_cut_rows(t, every[r][:, 0].copy(), np.ascontiguousarray(every[r][:, 1:]))
                got += every[r].shape[0]
        for t in (1, 0):
            marks[t] = eng.cuts_count(t)
        return got

    def rebalance(self, eng, sizes: Sequence[int]) -> int:
        """Work sharing while a shard is idle (see the module docstring); returns the
        records this shard received."""
        donors, idle = plan(sizes)
        if not donors:
            return 0
        mine = dict(donors).get(self.rank, 0)
        blob = pack_batch(eng.frontier_take(mine, from_bottom=True)) if mine else np.zeros(0, np.uint8)
        blobs = self.allgather_bytes(blob)
        if self.rank not in idle:
            return 0
        j = idle.index(self.rank)
        got = 0
        from .engine import batch_slice
        for r, g in donors:
            b = unpack_batch(blobs[r])
            lo = b.n * j // len(idle)
            hi = b.n * (j + 1) // len(idle)
            if hi > lo:
                eng.frontier_push(batch_slice(b, np.arange(lo, hi)))
                got += hi - lo
        return got


class LocalGroup:
    """Shared state of `world` frontier shards that run as threads of one process."""

    def __init__(self, world: int):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world


class LocalComm(ShardComm):
    """ShardComm's exchanges between threads of one process: several frontier shards on one
    GPU, each with its own device context (its own HIP stream and scratch), so that while one
    shard waits for the slowest record of its relaxation batch the others keep the GPU busy --
    the reference's several worker threads per node, each with its own NodeExplorer
    (DDSolver.cpp:684-760).  Same protocol as the multi-rank path: the collectives become a
    slot write per shard between two barriers."""

    def __init__(self, group: LocalGroup, rank: int):
        self.torch = None
        self.dist = None
        self.group = group
        self.world = group.world
        self.rank = rank
        self.dev = None
        self.bytes = 0

    def _exchange(self, value):
        g = self.group
        g.slots[self.rank] = value
        g.barrier.wait()
        out = list(g.slots)
        g.barrier.wait()
        return out

    def allreduce_max(self, z: float) -> float:
        self.bytes += 8
        return max(self._exchange(float(z)))

    def allgather_i64(self, vals: Sequence[int]) -> np.ndarray:
        self.bytes += 8 * len(vals)
        return np.stack([np.asarray(v, dtype=np.int64) for v in self._exchange([int(x) for x in vals])])

    def allgather_rows(self, rows: np.ndarray) -> List[np.ndarray]:
        rows = np.array(rows, dtype=np.float64, copy=True)
        self.bytes += rows.nbytes
        return self._exchange(rows)

    def allgather_bytes(self, blob: np.ndarray) -> List[np.ndarray]:
        blob = np.array(blob, dtype=np.uint8, copy=True)
        self.bytes += blob.nbytes
        return self._exchange(blob)


def run_local_shards(solvers, fn):
    """fn(solver) on every shard in its own thread (the library releases the GIL in its calls);
    returns the results in shard order, re-raising the first exception."""
    out = [None] * len(solvers)
    err = []

    def body(k):
        try:
            out[k] = fn(solvers[k])
        except BaseException as e:   # noqa: BLE001 -- re-raised below
            err.append(e)
            for s in solvers:        # unblock the other shards' barriers
                c = getattr(s, "comm", None)
                if c is not None and hasattr(c, "group"):
                    c.group.barrier.abort()
    threads = [threading.Thread(target=body, args=(k,)) for k in range(len(solvers))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if err:
        raise err[0]
    return out
