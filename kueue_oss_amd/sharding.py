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


_BUFS: dict = {}


def _exchange_buffers(key, words: int, world: int, dtype, device):
    """Reused exchange buffers for one (capacity, world, device): a pinned host
    staging row (async host-to-device copy), the device send row and the
    [world, words] receive block (RCCL all_gather_into_tensor).  Host
    collectives (gloo, device None / "cpu") send the host row itself."""
    import torch

    k = (key, words, world, str(device), dtype)
    b = _BUFS.get(k)
    if b is None:
        cuda = device is not None and str(device).startswith("cuda")
        host = torch.zeros(words, dtype=dtype, pin_memory=cuda)
        send = torch.empty(words, dtype=dtype, device=device) if cuda else host
        recv = torch.empty((world, words), dtype=dtype, device=device if cuda else None)
        for old in [x for x in _BUFS if x[0] == key]:  # one live capacity per exchange
            del _BUFS[old]
        b = _BUFS[k] = (host, send, recv, cuda)
    return b


def gather_assignments(quads, world: int, dist, device=None, to_host: bool = True):
    """All-gather every rank's full assignments (kueue_tas_host_last_assignments
    int32 quads: per workload a header and one (id, podset, leaf, count) per
    assigned domain) over RCCL (xGMI) or gloo.  Each rank sends one padded
    record row [length, quads..., padding] of the shared capacity from reused
    buffers (pinned staging, one async host-to-device copy; RCCL:
    all_gather_into_tensor into one [world, capacity] block); a round in which
    some rank's quads exceed the capacity is repeated once with a larger one
    (every rank sees every length, so all agree).  Returns the concatenated
    int32 numpy array, ranks in order (every rank receives all of it), or with
    ``to_host=False`` the device block and the per-rank lengths (no
    device-to-host copy of the block: a rank that does not admit).  That
    block is the exchange's reused receive buffer: it is valid until the next
    exchange (clone it to keep it); the lengths are a copy."""
    import numpy as np
    import torch

    q = np.ascontiguousarray(quads, dtype=np.int32).reshape(-1)
    n = q.size
    while True:
        cap = _CAP["gather"]
        host, send, recv, cuda = _exchange_buffers("gather", cap + 1, world, torch.int32, device)
        hv = host.numpy()
        hv[0] = n
        hv[1:1 + min(n, cap)] = q[:cap]  # words past the length are never read
        if cuda:
            send.copy_(host, non_blocking=True)  # ordered before the collective on the current stream
            dist.all_gather_into_tensor(recv, send)
        else:
            dist.all_gather(list(recv.unbind(0)), send)
        # (synchronizes: the staging row is free again); a copy, never a view of the reused block
        lens = np.array(recv[:, 0].cpu().numpy(), copy=True)
        if int(lens.max()) <= cap:
            if not to_host:
                return recv, lens
            parts = recv.cpu().numpy()  # the exchange's one device-to-host copy
            return np.concatenate([parts[r, 1:1 + int(lens[r])] for r in range(world)])
        _grow("gather", int(lens.max()))


def broadcast_deltas(deltas, dist, src: int = 0, device=None):
    """Broadcast the post-admission snapshot deltas (numpy
    native.DELTA_DTYPE records: leaf, column, int64 delta — updateTASUsage,
    tas_flavor_snapshot.go:257-293) from rank ``src``; every replica gets the
    identical list to apply with kueue_tas_host_apply_deltas.  One padded
    buffer [count, records as two int64 words each...] of the shared
    capacity (reused pinned staging and device row); a count of -1 is the
    source's failure sentinel (admit_round)."""
    import numpy as np
    import torch

    from .native import DELTA_DTYPE

    is_src = dist.get_rank() == src
    k = -1 if is_src and deltas is None else (len(deltas) if is_src else 0)
    while True:
        cap = _CAP["deltas"]
        host, buf, _, cuda = _exchange_buffers("deltas", 1 + 2 * cap, 1, torch.int64, device)
        hv = host.numpy()
        if is_src:
            hv[0] = k
            if 0 < k <= cap:
                hv[1:1 + 2 * k] = np.ascontiguousarray(deltas, dtype=DELTA_DTYPE).view(np.int64)
            if cuda:
                buf.copy_(host, non_blocking=True)
        dist.broadcast(buf, src)
        if cuda:
            host.copy_(buf)  # (synchronous: the records are read right away)
        got = hv
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
    Returns (gathered quads, admitted (id, 0/1) pairs or None off-src, deltas).
    Over RCCL the gathered block stays on the device: rank ``src`` admits
    from it (kueue_tas_host_admit_block: records and deltas built on the
    device, no host round trip of the quads) and the quads returned are None."""
    quads = block = lens = None
    if device is not None and str(device).startswith("cuda"):
        block, lens = gather_assignments(snap.last_assignments(), world, dist, device, to_host=False)
    else:
        quads = gather_assignments(snap.last_assignments(), world, dist, device)
    admitted = None
    deltas = None
    if rank == src:
        try:
            admitted, deltas = snap.admit(quads) if block is None else snap.admit_block(block, lens)
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
