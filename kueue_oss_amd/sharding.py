"""Data parallelism over pending workloads.

Every workload at the head of a queue is evaluated against the same
immutable snapshot (pkg/scheduler/scheduler.go:583-619), so the batch shards
across GPUs with the snapshot replicated; all PodSet groups of one workload
stay on one rank (assumedUsage chaining, tas_flavor_snapshot.go:543-591).
After the batch every rank's full assignments are all-gathered
(``gather_assignments``); rank 0 admits them in workload order and the
delta list it applied is broadcast to the other replicas (``admit_round``).
"""
from __future__ import annotations


def workload_cost(wl: list) -> float:
    """Relative device cost of a workload: unconstrained/implied requests
    scan the leaf level; multi-group workloads need extra passes."""
    c = 0.0
    for p in wl:
        tr = p.get("topologyRequest")
        c += 4.0 if tr is None or tr.get("unconstrained") else 1.0
    return c


def shard_ids(workloads: list, world: int, rank: int) -> list:
    """Global indices of rank's cost-balanced, deterministic shard (greedy
    longest-processing-time on the global order; identical on every rank),
    in ascending order."""
    if world <= 1:
        return list(range(len(workloads)))
    import heapq

    heap = [(0.0, k) for k in range(world)]
    order = sorted(range(len(workloads)), key=lambda i: (-workload_cost(workloads[i]), i))
    assign = [0] * len(workloads)
    for i in order:
        load, r = heapq.heappop(heap)
        assign[i] = r
        heapq.heappush(heap, (load + workload_cost(workloads[i]), r))
    return [i for i in range(len(workloads)) if assign[i] == rank]


def shard_workloads(workloads: list, world: int, rank: int) -> list:
    """The workloads of ``shard_ids``."""
    return [workloads[i] for i in shard_ids(workloads, world, rank)]


# Fixed-capacity exchange buffers (in int32 / int64 words), remembered across
# rounds and grown to the next power of two when a round overflows them: in
# the steady state one collective and one device-to-host copy per exchange,
# no size round trip and no per-rank .item() syncs.
_CAP = {"gather": 1 << 16, "deltas": 1 << 12}


def _grow(key, need):
    c = _CAP[key]
    while c < need:
        c *= 2
    _CAP[key] = c
    return c


def gather_assignments(quads, world: int, dist, device=None):
    """All-gather every rank's full assignments (kueue_tas_host_last_assignments
    int32 quads: per workload a header and one (id, podset, leaf, count) per
    assigned domain) over RCCL (xGMI) or gloo.  Each rank sends one padded
    record buffer [length, quads..., padding] of the shared capacity; a round
    in which some rank's quads exceed it is repeated once with a larger
    capacity (every rank sees every length, so all agree).  Returns the
    concatenated int32 numpy array, ranks in order; every rank receives all of it."""
    import numpy as np
    import torch

    q = np.ascontiguousarray(quads, dtype=np.int32).reshape(-1)
    n = q.size
    while True:
        cap = _CAP["gather"]
        host = np.zeros(cap + 1, dtype=np.int32)
        host[0] = n
        host[1:1 + min(n, cap)] = q[:cap]
        buf = torch.from_numpy(host).to(device)
        out = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(out, buf)
        parts = torch.stack(out).cpu().numpy()  # the exchange's one device-to-host copy
        lens = parts[:, 0]
        if int(lens.max()) <= cap:
            return np.concatenate([parts[r, 1:1 + int(lens[r])] for r in range(world)])
        _grow("gather", int(lens.max()))


def broadcast_deltas(deltas, dist, src: int = 0, device=None):
    """Broadcast the post-admission snapshot deltas (numpy
    native.DELTA_DTYPE records: leaf, column, int64 delta — updateTASUsage,
    tas_flavor_snapshot.go:257-293) from rank ``src``; every replica gets the
    identical list to apply with kueue_tas_host_apply_deltas.  One padded
    buffer [count, records as two int64 words each...] of the shared
    capacity; a count of -1 is the source's failure sentinel (admit_round)."""
    import numpy as np
    import torch

    from .native import DELTA_DTYPE

    is_src = dist.get_rank() == src
    k = -1 if is_src and deltas is None else (len(deltas) if is_src else 0)
    while True:
        cap = _CAP["deltas"]
        host = np.zeros(1 + 2 * cap, dtype=np.int64)
        if is_src:
            host[0] = k
            if 0 < k <= cap:
                host[1:1 + 2 * k] = np.ascontiguousarray(deltas, dtype=DELTA_DTYPE).view(np.int64)
        buf = torch.from_numpy(host).to(device)
        dist.broadcast(buf, src)
        got = buf.cpu().numpy()
        k = int(got[0])
        if k < 0:  # the source's admission failed: every rank fails with it
            raise RuntimeError(f"admission failed on rank {src}")
        if k <= cap:
            return got[1:1 + 2 * k].copy().view(DELTA_DTYPE)
        _grow("deltas", k)


def admit_round(snap, world: int, rank: int, dist, device=None, src: int = 0):
    """One nominate/admit round after every rank's run_compiled: all-gather the
    assignments, rank ``src`` admits in workload order (Fits + AddUsage on its
    replica) and broadcasts the applied deltas, the other replicas apply them.
    Returns (gathered quads, admitted (id, 0/1) pairs or None off-src, deltas)."""
    quads = gather_assignments(snap.last_assignments(), world, dist, device)
    admitted = None
    deltas = None
    if rank == src:
        try:
            admitted, deltas = snap.admit(quads)
        except Exception:
            # a failed admission must not leave the other ranks waiting in the
            # broadcast: send the failure count (-1) so every rank raises
            try:
                broadcast_deltas(None, dist, src, device)
            except RuntimeError:
                pass  # the sentinel's own echo; the original error propagates
            raise
    deltas = broadcast_deltas(deltas, dist, src, device)
    if rank != src:
        snap.apply_deltas(deltas)
    return quads, admitted, deltas
