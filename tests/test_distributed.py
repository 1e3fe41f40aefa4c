"""Multi-rank path on CPU (gloo, world_size 2): cost-balanced sharding keeps
every workload on exactly one rank, result records all-gather, and the
admission delta list broadcasts identically to every replica."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kueue_oss_amd import sharding, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _, wls = synth.config_c2(n_workloads=50)
    mine = sharding.shard_workloads(wls, world, rank)
    # per-workload records: [global index, #podsets, 0, 0]
    idx = {id(w): i for i, w in enumerate(wls)}
    recs = []
    for w in mine:
        recs += [idx[id(w)], len(w), 0, 0]
    got = sharding.gather_records(recs, world, dist)
    deltas = [(3, 1, 1000), (7, 0, -5)] if rank == 0 else None
    bd = sharding.broadcast_deltas(deltas, dist, src=0)
    q.put((rank, got, bd))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_shard_gather_broadcast(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    gathered = out[0][1]
    assert gathered == out[1][1]
    seen = sorted(r[i] for r in gathered for i in range(0, len(r), 4))
    assert seen == list(range(50))  # each workload on exactly one rank
    assert out[0][2] == out[1][2] == [(3, 1, 1000), (7, 0, -5)]


def test_shard_is_cost_balanced():
    _, wls = synth.config_c2(n_workloads=400)
    shards = [sharding.shard_workloads(wls, 4, r) for r in range(4)]
    assert sum(len(s) for s in shards) == 400
    loads = [sum(sharding.workload_cost(w) for w in s) for s in shards]
    assert max(loads) - min(loads) <= 4.0
