"""Full-size GPU parity: the benched batches as a whole, and the sharded
multi-rank path with two ranks on the one GPU of the box.

* C3 (131,072 nodes) and C3J (ragged racks, ~1,000 phase-1 classes): every
  one of the 1,024 workloads of the bench step (the same flags: compile +
  evaluation + TopologyAssignment values, ``RUN_COMPILE | RUN_VALUES``)
  against a 16-thread oracle run.
* C5 (1,048,576 nodes): two ranks, each evaluating its cost-balanced shard of
  a 2,048-workload batch (1,024 per rank, ``max_batch=1024``) through
  ``shard_ids`` + ``run_compiled`` + ``gather_assignments`` + ``admit_round``
  (gloo collectives over host tensors: RCCL needs one GPU per rank), then a
  second batch on the updated replicas.  Checked against (a) one unsharded
  replica on the same GPU running the same sequence (every assignment, every
  admission decision, every delta, the whole second batch), (b) the oracle:
  a stratified sample of both batches, and every admission decision replayed
  as Fits + AddUsage in workload order on the oracle snapshot
  (scheduler.go:371-435, tas_flavor_snapshot.go:401-415, :257-293).
"""
import os
import socket
import sys
import threading
import time

import numpy as np
import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, sharding, synth

pytestmark = pytest.mark.gpu
FULL = TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES


def _whole_batch(gen, n=1024):
    doc, wls = gen(n_workloads=n)
    snap = TASFlavorSnapshot(doc)
    snap.compile(wls)
    snap.run_compiled(flags=FULL)
    got = snap.last_results()
    snap.close()
    want, _ = oracle_lib.eval_workloads(doc, wls, threads=16)
    mism = [i for i in range(len(wls)) if got[i] != want[i]]
    assert mism == [], (len(mism), mism[:8])
    return got


@pytest.mark.timeout(600)
def test_c3_whole_batch_on_gpu():
    got = _whole_batch(synth.config_c3)
    assert sum(1 for r in got if all(not p["reason"] for p in r)) > 500


@pytest.mark.timeout(600)
def test_c3j_whole_batch_on_gpu():
    got = _whole_batch(synth.config_c3j)
    assert sum(1 for r in got if all(not p["reason"] for p in r)) > 500


# ---- C5 sharded over two ranks on one GPU ----
C5_PER_RANK = 1024
WORLD = 2


_CAPFD = None  # the running test's capfd: progress goes to the terminal past pytest's capture


def _progress(msg):
    line = f"[c5] {time.strftime('%H:%M:%S')} {msg}"
    if _CAPFD is not None:
        with _CAPFD.disabled():
            print(line, file=sys.stderr, flush=True)
    else:
        print(line, file=sys.stderr, flush=True)


def _heartbeat(stop, period=20.0):
    """Progress lines while the 1M-node phases run (setup and the oracle print
    nothing), so a runner that takes a silent minute for a hang sees it alive."""
    t0 = time.time()
    while not stop.wait(period):
        _progress(f"alive {time.time() - t0:.0f}s")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sample_ids(wls, ids, k=8):
    """k BestFit (required / preferred) and k unconstrained workloads of a shard."""
    bf = [i for i in ids if wls[i][0]["topologyRequest"] and not wls[i][0]["topologyRequest"].get("unconstrained")]
    lfc = [i for i in ids if i not in set(bf)]
    return bf[:k] + lfc[:k]


def _c5():
    return synth.config_c5(n_workloads=C5_PER_RANK * WORLD)


def _rank_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        doc, wls = _c5()
        ids = sharding.shard_ids(wls, world, rank)
        snap = TASFlavorSnapshot(doc, device=0, max_batch=C5_PER_RANK)
        del doc
        snap.compile(wls)
        snap.set_shard(ids)
        out = {"ids": ids}
        snap.run_compiled(flags=FULL)
        res = snap.last_results()
        pos = {g: k for k, g in enumerate(ids)}
        out["sample1"] = {i: res[pos[i]] for i in _sample_ids(wls, ids, 4)}
        out["gathered1"] = sharding.gather_assignments(snap.last_assignments(), world, dist)
        quads, admitted, deltas = sharding.admit_round(snap, world, rank, dist)
        out["admit_quads"] = quads
        out["admitted"] = admitted
        out["deltas"] = deltas
        snap.run_compiled(flags=FULL)
        res = snap.last_results()
        out["sample2"] = {i: res[pos[i]] for i in _sample_ids(wls, ids, 4)}
        out["gathered2"] = sharding.gather_assignments(snap.last_assignments(), world, dist)
        snap.close()
        q.put((rank, out))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, {"error": repr(e)}))
        raise
    finally:
        dist.destroy_process_group()


def _by_workload(quads):
    """{workload id: (failed, sorted (podset, leaf, count) records)} of gathered quads."""
    q = np.asarray(quads, dtype=np.int32).reshape(-1, 4)
    out = {}
    for g, p, leaf, c in q.tolist():
        if p < 0:
            out.setdefault(g, [leaf, []])[0] = leaf  # header: (id, -1, failed, n)
        else:
            out.setdefault(g, [0, []])[1].append((p, leaf, c))
    return {g: (f, sorted(r)) for g, (f, r) in out.items()}


@pytest.mark.timeout(1200)
def test_c5_sharded_two_ranks_on_one_gpu(capfd):
    global _CAPFD
    _CAPFD = capfd
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(stop,), daemon=True).start()
    try:
        _c5_sharded()
    finally:
        stop.set()
        _CAPFD = None


def _c5_sharded():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=900) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=120)
    for r in range(WORLD):
        assert "error" not in outs[r], outs[r].get("error")
        assert procs[r].exitcode == 0
    _progress("ranks done")
    doc, wls = _c5()
    n = len(wls)
    assert sorted(i for r in range(WORLD) for i in outs[r]["ids"]) == list(range(n))
    assert all(len(outs[r]["ids"]) <= C5_PER_RANK + 64 for r in range(WORLD))
    for key in ("gathered1", "gathered2", "admit_quads"):
        assert np.array_equal(outs[0][key], outs[1][key]), key
    assert outs[0]["deltas"].tolist() == outs[1]["deltas"].tolist()
    g1, g2 = _by_workload(outs[0]["gathered1"]), _by_workload(outs[0]["gathered2"])
    assert sorted(g1) == list(range(n)) and sorted(g2) == list(range(n))

    # (a) one unsharded replica on the same GPU, same sequence
    snap = TASFlavorSnapshot(doc, max_batch=C5_PER_RANK)
    snap.compile(wls)
    snap.run_compiled(flags=FULL)
    u1 = _by_workload(snap.last_assignments())
    admitted, deltas = snap.admit(snap.last_assignments())
    snap.run_compiled(flags=FULL)
    u2 = _by_workload(snap.last_assignments())
    leaf_names = snap.leaf_ids()
    snap.close()
    assert [w for w in range(n) if g1[w] != u1[w]] == []
    assert outs[0]["admitted"].tolist() == admitted.tolist()
    assert np.array_equal(np.sort(outs[0]["deltas"], order=["leaf", "col"]), np.sort(deltas, order=["leaf", "col"]))
    assert [w for w in range(n) if g2[w] != u2[w]] == []
    n_adm = int(admitted[:, 1].sum())
    assert 0 < n_adm < n

    _progress("unsharded replica agrees")
    # (b) the oracle: batch-1 sample, every admission decision, batch-2 sample
    s1 = {i: r for o in outs.values() for i, r in o["sample1"].items()}
    ids1 = sorted(s1)
    want1, _ = oracle_lib.eval_workloads(doc, [wls[i] for i in ids1], threads=16)
    assert [i for k, i in enumerate(ids1) if s1[i] != want1[k]] == []

    def usage(w):  # ComputeTASNetUsage records from the gathered quads (lowest level: hostname)
        recs = []
        for p, leaf, c in g1[w][1]:
            req = wls[w][p].get("requests", {})
            recs.append({"values": [leaf_names[leaf]], "singlePodRequests": dict(req), "count": c})
        return recs

    _progress("oracle batch-1 sample agrees")
    cand = [w for w in range(n) if not g1[w][0]]
    s2 = {i: r for o in outs.values() for i, r in o["sample2"].items()}
    ids2 = sorted(s2)
    ops = [{"op": "admit", "usage": usage(w)} for w in cand]
    ops += [{"op": "find", "podSets": wls[i]} for i in ids2]
    res = oracle_lib.session(doc, ops)
    got_adm = dict(admitted.tolist())
    assert {w: bool(got_adm[w]) for w in cand} == dict(zip(cand, res[:len(cand)]))
    assert all(not got_adm[w] for w in range(n) if g1[w][0])
    assert [i for k, i in enumerate(ids2) if s2[i] != res[len(cand) + k]] == []
