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


def _gather_var(arr, world: int, dist, device=None):
    """All-gather a variable-length 1-D tensor: sizes first, then the buffers
    padded to the largest (RCCL / gloo all_gather need equal shapes)."""
    import torch

    n = torch.tensor([arr.numel()], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = max(int(x.item()) for x in sizes)
    pad = torch.zeros((max(m, 1),), dtype=arr.dtype, device=device)
    pad[: arr.numel()] = arr
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad)
    return [o[: int(sizes[i].item())] for i, o in enumerate(out)]


def gather_assignments(quads, world: int, dist, device=None):
    """All-gather every rank's full assignments (kueue_tas_host_last_assignments
    int32 quads: per workload a header and one (id, podset, leaf, count) per
    assigned domain) over RCCL (xGMI) or gloo.  Returns the concatenated int32
    numpy array, ranks in order; every rank receives all of it."""
    import numpy as np
    import torch

    t = torch.from_numpy(np.ascontiguousarray(quads, dtype=np.int32)).to(device)
    parts = _gather_var(t, world, dist, device)
    return torch.cat(parts).cpu().numpy() if parts else np.zeros(0, dtype=np.int32)


def broadcast_deltas(deltas, dist, src: int = 0, device=None):
    """Broadcast the post-admission snapshot deltas (numpy
    native.DELTA_DTYPE records: leaf, column, int64 delta — updateTASUsage,
    tas_flavor_snapshot.go:257-293) from rank ``src``; every replica gets the
    identical list to apply with kueue_tas_host_apply_deltas."""
    import numpy as np
    import torch

    from .native import DELTA_DTYPE

    is_src = dist.get_rank() == src
    n = torch.tensor([len(deltas) if is_src and deltas is not None else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    k = int(n.item())
    if k < 0:  # the source's admission failed (admit_round): every rank fails with it
        raise RuntimeError(f"admission failed on rank {src}")
    if k == 0:
        return np.zeros(0, dtype=DELTA_DTYPE)
    if is_src:  # 16-byte records as two int64 words
        words = np.ascontiguousarray(deltas, dtype=DELTA_DTYPE).view(np.int64).reshape(k, 2)
        buf = torch.from_numpy(words.copy()).to(device)
    else:
        buf = torch.zeros((k, 2), dtype=torch.int64, device=device)
    dist.broadcast(buf, src)
    return buf.cpu().numpy().reshape(-1).view(DELTA_DTYPE).copy()


def admit_round(snap, world: int, rank: int, dist, device=None, src: int = 0):
    """One nominate/admit round after every rank's run_compiled: all-gather the
    assignments, rank ``src`` admits in workload order (Fits + AddUsage on its
    replica) and broadcasts the applied deltas, the other replicas apply them.
    Returns (gathered quads, admitted (id, 0/1) pairs or None off-src, deltas)."""
    import torch

    quads = gather_assignments(snap.last_assignments(), world, dist, device)
    admitted = None
    deltas = None
    if rank == src:
        try:
            admitted, deltas = snap.admit(quads)
        except Exception:
            # a failed admission must not leave the other ranks waiting in the
            # broadcast: send the failure count (-1) so every rank raises
            dist.broadcast(torch.tensor([-1], dtype=torch.int64, device=device), src)
            raise
    deltas = broadcast_deltas(deltas, dist, src, device)
    if rank != src:
        snap.apply_deltas(deltas)
    return quads, admitted, deltas
