"""Multi-rank path on CPU (gloo, world_size 2).

Each rank holds a replica of the snapshot (here the emulated build of the
product library, tests/emu), compiles the same global workload list and
evaluates its cost-balanced shard; the full assignments are all-gathered,
rank 0 admits in workload order (Fits + AddUsage: the TAS half of
processEntry, pkg/scheduler/scheduler.go:371-435) and broadcasts the delta
list it applied, the other replica applies it; a second batch then runs on
the updated replicas.  Every assignment and admission decision must equal the
oracle session: find every workload, admit them in order, find again."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kueue_oss_amd import sharding, synth

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload(n=40):
    return synth.config_c2(n_workloads=n, shape=(2, 2, 8, 16))


def _worker(rank, world, port, q, lib_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kueue_oss_amd import TASFlavorSnapshot, native

        lib = native.load_library(lib_path)
        snap_doc, wls = _workload()
        ids = sharding.shard_ids(wls, world, rank)
        snap = TASFlavorSnapshot(snap_doc, lib=lib)
        snap.compile(wls)
        snap.set_shard(ids)
        out = {"ids": ids}
        snap.run_compiled()
        out["batch1"] = snap.last_results()
        quads, admitted, deltas = sharding.admit_round(snap, world, rank, dist)
        out["quads"] = quads.tolist()
        out["admitted"] = admitted.tolist() if admitted is not None else None
        out["deltas"] = deltas.tolist()
        snap.run_compiled()
        out["batch2"] = snap.last_results()
        snap.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_shard_gather_admit_broadcast(world, emu_lib):
    import oracle_lib

    lib_path = os.path.join(HERE, "emu", "_build", "libkueue_tas_emu.so")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, lib_path)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    snap_doc, wls = _workload()
    n = len(wls)
    # every workload on exactly one rank
    assert sorted(i for r in range(world) for i in outs[r]["ids"]) == list(range(n))
    # identical gathered assignments and deltas everywhere
    assert outs[0]["quads"] == outs[1]["quads"]
    assert outs[0]["deltas"] == outs[1]["deltas"]

    def by_id(key):
        res = {}
        for r in range(world):
            for i, rs in zip(outs[r]["ids"], outs[r][key]):
                res[i] = rs
        return [res[i] for i in range(n)]

    b1, b2 = by_id("batch1"), by_id("batch2")
    # the oracle session: find all, admit in order the ones without failure, find all again
    ops = [{"op": "find", "podSets": w} for w in wls]
    admit_idx = []
    for i, w in enumerate(wls):
        if all(not r["reason"] for r in b1[i]):
            ops.append({"op": "admit", "usage": synth.usage_records(w, b1[i])})
            admit_idx.append(i)
    ops += [{"op": "find", "podSets": w} for w in wls]
    res = oracle_lib.session(snap_doc, ops)
    assert b1 == res[:n]
    want_admit = dict(zip(admit_idx, res[n:n + len(admit_idx)]))
    got_admit = {int(i): bool(a) for i, a in outs[0]["admitted"]}
    assert {i: got_admit[i] for i in want_admit} == want_admit
    assert all(not got_admit[i] for i in range(n) if i not in want_admit)
    assert any(want_admit.values()) and not all(want_admit.values())
    assert b2 == res[n + len(admit_idx):]


def _failing_worker(rank, world, port, q, lib_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kueue_oss_amd import TASFlavorSnapshot, native

        lib = native.load_library(lib_path)
        snap_doc, wls = _workload(8)
        snap = TASFlavorSnapshot(snap_doc, lib=lib)
        snap.compile(wls)
        snap.set_shard(sharding.shard_ids(wls, world, rank))
        snap.run_compiled()
        if rank == 0:
            def broken_admit(quads):
                raise RuntimeError("forced admission failure")

            snap.admit = broken_admit
        try:
            sharding.admit_round(snap, world, rank, dist)
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, str(e)))
        snap.close()
    finally:
        dist.destroy_process_group()


def test_admit_failure_fails_every_rank(emu_lib):
    """A host error in rank 0's admission: every rank raises
    instead of the others waiting forever in the delta broadcast."""
    lib_path = os.path.join(HERE, "emu", "_build", "libkueue_tas_emu.so")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, 2, port, q, lib_path)) for r in range(2)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert outs[0] == "forced admission failure"
    assert outs[1] == "admission failed on rank 0"


def test_shard_is_cost_balanced():
    _, wls = synth.config_c2(n_workloads=400)
    shards = [sharding.shard_workloads(wls, 4, r) for r in range(4)]
    assert sum(len(s) for s in shards) == 400
    loads = [sum(sharding.workload_cost(w) for w in s) for s in shards]
    assert max(loads) - min(loads) <= 4.0
    ids = [sharding.shard_ids(wls, 4, r) for r in range(4)]
    assert sorted(i for s in ids for i in s) == list(range(400))
    assert [[wls[i] for i in s] for s in ids] == shards


def test_delta_records_roundtrip():
    from kueue_oss_amd.native import DELTA_DTYPE

    d = np.zeros(3, dtype=DELTA_DTYPE)
    d["leaf"] = [1, 2, 3]
    d["col"] = [0, 4, 2]
    d["delta"] = [-5, 1 << 40, 7]
    words = d.view(np.int64).reshape(3, 2)
    assert words.reshape(-1).view(DELTA_DTYPE).tolist() == d.tolist()


_NCCL_EXCHANGE = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from kueue_oss_amd import sharding
from kueue_oss_amd.native import DELTA_DTYPE

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
rng = np.random.default_rng(5)
for n in (12, 4 * 70000):  # the second overflows the initial capacity: the grow-and-repeat round
    q = rng.integers(-5, 1 << 20, size=n, dtype=np.int32)
    got = sharding.gather_assignments(q, 1, dist, "cuda:0")
    assert np.array_equal(got, q), n
    block, lens = sharding.gather_assignments(q, 1, dist, "cuda:0", to_host=False)
    assert block.is_cuda and int(lens[0]) == n
    assert np.array_equal(block[0, 1:1 + n].cpu().numpy(), q)
d = np.zeros(5000, dtype=DELTA_DTYPE)  # overflows the initial delta capacity
d["leaf"] = np.arange(5000)
d["col"] = 1
d["delta"] = -(np.arange(5000, dtype=np.int64) << 33)
got = sharding.broadcast_deltas(d, dist, 0, "cuda:0")
assert np.array_equal(got, d)
# admit_round over RCCL: rank 0 admits from the gathered device block
# (kueue_tas_host_admit_block); the same verdicts and deltas as the host path
from kueue_oss_amd import TASFlavorSnapshot, synth
doc, wls = synth.config_c2(n_workloads=256, shape=(2, 4, 8, 16))
ref = TASFlavorSnapshot(doc)
ref.compile(wls)
ref.run_compiled()
want_adm, want_d = ref.admit(ref.last_assignments())
ref.close()
snap = TASFlavorSnapshot(doc)
snap.compile(wls)
snap.run_compiled()
quads, adm, dl = sharding.admit_round(snap, 1, 0, dist, "cuda:0")
assert quads is None and np.array_equal(adm, want_adm) and np.array_equal(dl, want_d)
assert 0 < int(adm[:, 1].sum()) < len(wls)
snap.close()
dist.destroy_process_group()
print("exchange ok")
"""


@pytest.mark.gpu
def test_exchange_buffers_on_rccl():
    """The RCCL side of the exchange (pinned staging, all_gather_into_tensor,
    device-resident block, capacity growth, delta broadcast, and admit_round
    admitting from the device block) in a one-rank nccl group on the box's
    GPU (a child process: its own process group)."""
    import subprocess
    import sys

    r = subprocess.run([sys.executable, "-c", _NCCL_EXCHANGE, os.path.dirname(HERE), str(_free_port())],
                       capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0 and "exchange ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
