"""Data parallelism over pending workloads.

Every workload at the head of a queue is evaluated against the same
immutable snapshot (pkg/scheduler/scheduler.go:583-619), so the batch shards
across GPUs with the snapshot replicated; all PodSet groups of one workload
stay on one rank (assumedUsage chaining, tas_flavor_snapshot.go:543-591).
After the batch, rank-local result records are all-gathered and the
admission delta list is broadcast (``broadcast_deltas``).
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


def shard_workloads(workloads: list, world: int, rank: int) -> list:
    """Cost-balanced, deterministic shard (greedy longest-processing-time on
    the global order; identical on every rank)."""
    if world <= 1:
        return list(workloads)
    loads = [0.0] * world
    owner = []
    order = sorted(range(len(workloads)), key=lambda i: (-workload_cost(workloads[i]), i))
    assign = [0] * len(workloads)
    for i in order:
        r = min(range(world), key=lambda k: (loads[k], k))
        loads[r] += workload_cost(workloads[i])
        assign[i] = r
    for i, w in enumerate(workloads):
        if assign[i] == rank:
            owner.append(w)
    return owner


def gather_records(records, world: int, dist, device=None):
    """All-gather fixed-size int32 result records ([n][4] per rank, padded to
    the max n) — RCCL on GPUs, gloo on CPU.  Returns the list of per-rank lists."""
    import torch

    t = torch.tensor(records, dtype=torch.int32, device=device)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(s.item() for s in sizes))
    pad = torch.full((m,), -1, dtype=torch.int32, device=device)
    pad[: t.numel()] = t
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad)
    return [o[: int(sizes[i].item())].tolist() for i, o in enumerate(out)]


def broadcast_deltas(deltas, dist, src: int = 0, device=None):
    """Broadcast the post-admission snapshot delta list [(leaf, col, delta)]
    from rank ``src`` so every replica applies the same usage change
    (updateTASUsage, tas_flavor_snapshot.go:257-293)."""
    import torch

    n = torch.tensor([len(deltas) if deltas is not None else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    k = int(n.item())
    buf = torch.zeros((k, 3), dtype=torch.int64, device=device)
    if dist.get_rank() == src and k:
        buf[:] = torch.tensor(deltas, dtype=torch.int64, device=device)
    dist.broadcast(buf, src)
    return [tuple(int(x) for x in row) for row in buf.tolist()]
