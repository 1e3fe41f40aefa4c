"""Snapshot usage updates (ClusterQueueSnapshot.AddUsage/RemoveUsage ->
updateTASUsage, clusterqueue_snapshot.go:94-119) and the admission re-check
(TASFlavorSnapshot.Fits, tas_flavor_snapshot.go:401-415), interleaved with
evaluations, against the oracle's restatement of the same session.  The
reference's tests hold no golden vector for Fits/updateTASUsage alone; the
usage arithmetic is the one the find goldens pin through `tasUsage`."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth


def _sessions(seed, n, lib=None, gen=None):
    rng = random.Random(seed)
    for i in range(n):
        case = (gen or synth.random_case)(rng)
        first = oracle_lib.run_case(case)["results"]
        ops = synth.admission_ops(rng, case, first)
        want = oracle_lib.session(case, ops)
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        got = synth.run_session(snap, ops)
        snap.close()
        for k, (g, w) in enumerate(zip(got, want)):
            assert g == w, (i, k, ops[k]["op"], g, w)


def test_oracle_session_replays_usage():
    # add then remove of the same records restores every evaluation
    rng = random.Random(3)
    for _ in range(20):
        case = synth.random_case(rng)
        first = oracle_lib.run_case(case)["results"]
        u = synth.usage_records(case["podSets"], first)
        ops = [{"op": "find", "podSets": case["podSets"]}, {"op": "add", "usage": u},
               {"op": "remove", "usage": u}, {"op": "find", "podSets": case["podSets"]}]
        r = oracle_lib.session(case, ops)
        assert r[0] == r[3] == first


@pytest.mark.parametrize("seed", [51, 52])
def test_emulated_admission_session(emu_lib, seed):  # noqa: F811
    _sessions(seed, 60, lib=emu_lib)


def test_emulated_admission_session_arith(emu_lib):  # noqa: F811
    _sessions(53, 40, lib=emu_lib, gen=synth.arith_stress_case)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [61, 62])
def test_admission_session_on_gpu(seed):
    _sessions(seed, 150)


@pytest.mark.gpu
def test_admission_session_arith_on_gpu():
    _sessions(63, 150, gen=synth.arith_stress_case)


def _admit_then_rebuild(make_snap, mode):
    """kueue_tas_host_admit applies usage on the device and defers the host
    mirror; a node event that re-assembles the snapshot must see every
    admitted record (the oracle rebuilt from a document holding that usage):
    a splice of a new leaf ("splice"), a second node under an existing
    hostname (capacity only, in place: "same-host"), and a rebuild (an update
    of the first node of such a hostname, whose taints and labels are the
    leaf's: "rebuild")."""
    import copy

    snap_doc, wls = synth.config_c2(n_workloads=24, shape=(2, 2, 4, 8))
    snap = make_snap(snap_doc)
    snap.compile(wls)
    snap.run_compiled()
    res = snap.last_results()
    admitted, deltas = snap.admit(snap.last_assignments())
    assert len(deltas) and admitted[:, 1].any()
    want_doc = copy.deepcopy(snap_doc)
    for i, ok in admitted.tolist():
        if ok:
            want_doc.setdefault("tasUsage", []).extend(synth.usage_records(wls[i], res[i]))
    extra = copy.deepcopy(snap_doc["nodes"][0])
    extra["name"] = "added-node"
    if mode == "splice":  # a node with a new rack: spliced into the tree in place
        for k in list(extra["labels"]):
            if k != "kubernetes.io/hostname":
                extra["labels"][k] = extra["labels"][k] + "-x"
        extra["labels"]["kubernetes.io/hostname"] = "added-node"
    # else: the first node's hostname — leafDomain.node stays the first node
    want_doc["nodes"].append(extra)
    c0 = snap.snapshot_counters()
    assert snap.update_nodes([extra]) is False
    assert snap.snapshot_counters()[0] == c0[0]  # no device reload
    if mode == "rebuild":
        first = copy.deepcopy(snap_doc["nodes"][0])
        first["labels"]["extra-label"] = "x"
        want_doc["nodes"][0] = first
        assert snap.update_nodes([first]) is True
    got = snap.find_topology_assignments_for_workloads(wls)
    snap.close()
    want, _ = oracle_lib.eval_workloads(want_doc, wls, threads=4)
    assert got == want


@pytest.mark.parametrize("mode", ["splice", "same-host", "rebuild"])
def test_emulated_admit_then_rebuild(emu_lib, mode):  # noqa: F811
    _admit_then_rebuild(lambda d: TASFlavorSnapshot(d, lib=emu_lib), mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["splice", "same-host", "rebuild"])
def test_admit_then_rebuild_on_gpu(mode):
    _admit_then_rebuild(lambda d: TASFlavorSnapshot(d), mode)


def _admit_relayout_apply(make_snap):
    """Replica deltas after a relayout: an admission leaves the
    device ahead of the host mirror; a node update with a new label key makes
    the device layout stale (the next upload reloads from the mirror); the
    negated admission deltas then arrive as another rank's delta list
    (kueue_tas_host_apply_deltas) and must survive the reload on every entry
    the admission touched.  The usage is back to the document's, so the
    oracle is the document with the node's new label."""
    import copy

    snap_doc, wls = synth.config_c2(n_workloads=24, shape=(2, 2, 4, 8))
    snap = make_snap(snap_doc)
    snap.compile(wls)
    snap.run_compiled()
    before = snap.last_results()
    admitted, deltas = snap.admit(snap.last_assignments())
    assert len(deltas) and admitted[:, 1].any()
    want_doc = copy.deepcopy(snap_doc)
    node = want_doc["nodes"][3]
    node["labels"]["example.com/brand-new-label"] = "x"
    assert snap.update_nodes([copy.deepcopy(node)]) is False  # in place, the device layout is stale
    neg = deltas.copy()
    neg["delta"] = -neg["delta"]
    snap.apply_deltas(neg)
    got = snap.find_topology_assignments_for_workloads(wls)
    snap.close()
    want, _ = oracle_lib.eval_workloads(want_doc, wls, threads=4)
    assert got == want
    assert got == before  # the label changes no request's fit


def test_emulated_admit_relayout_apply(emu_lib):  # noqa: F811
    _admit_relayout_apply(lambda d: TASFlavorSnapshot(d, lib=emu_lib))


@pytest.mark.gpu
def test_admit_relayout_apply_on_gpu():
    _admit_relayout_apply(lambda d: TASFlavorSnapshot(d))


def _usage_updates_after_admission(make_snap):
    """AddUsage / RemoveUsage (kueue_tas_host_update_usage) right after a
    device admission: the admission stays pending on the mirror (no diff of
    the whole usage), the update reaches the device, the mirror and its
    shadow; a later reader (free capacity) sees both.  Against the oracle
    session: admit, add a record list, remove another, find."""
    snap_doc, wls = synth.config_c2(n_workloads=24, shape=(2, 2, 4, 8))
    snap = make_snap(snap_doc)
    snap.compile(wls)
    snap.run_compiled()
    b1 = snap.last_results()
    admitted, _ = snap.admit(snap.last_assignments())
    ok = [i for i, a in admitted.tolist() if a]
    assert len(ok) >= 3
    add = synth.usage_records(wls[ok[0]], b1[ok[0]])
    rem = synth.usage_records(wls[ok[1]], b1[ok[1]])
    snap.add_usage(add)
    snap.remove_usage(rem)
    got = snap.find_topology_assignments_for_workloads(wls)
    free = snap.serialize_free_capacity_per_domain()
    lib = snap._lib
    snap.close()
    ops = [{"op": "add", "usage": synth.usage_records(wls[i], b1[i])} for i in ok]
    ops += [{"op": "add", "usage": add}, {"op": "remove", "usage": rem}]
    ops += [{"op": "find", "podSets": w} for w in wls]
    assert got == oracle_lib.session(snap_doc, ops)[len(ok) + 2:]
    # the host mirror equals one that took the same usage through AddUsage only
    ref = TASFlavorSnapshot(snap_doc, lib=lib)
    for op in ops[:len(ok) + 2]:
        (ref.add_usage if op["op"] == "add" else ref.remove_usage)(op["usage"])
    assert free == ref.serialize_free_capacity_per_domain()
    ref.close()


def test_emulated_usage_updates_after_admission(emu_lib):  # noqa: F811
    _usage_updates_after_admission(lambda d: TASFlavorSnapshot(d, lib=emu_lib))


@pytest.mark.gpu
def test_usage_updates_after_admission_on_gpu():
    _usage_updates_after_admission(lambda d: TASFlavorSnapshot(d))


def _admit_batch(make, n=64, shape=(2, 2, 4, 8), huge_memory=False):
    """kueue_tas_host_admit over one evaluated batch (admit_fit0_kernel +
    admit_kernel: phase-1 rejections, re-checks of workloads whose leaves an
    earlier admission touched) against the oracle session: find every
    workload, admit in order the ones that found an assignment, find again."""
    snap_doc, wls = synth.config_c2(n_workloads=n, shape=shape)
    if huge_memory:  # capacities of 2^62: the limits' preconditions fail, the exact re-check pass runs
        for nd in snap_doc["nodes"]:
            nd["allocatable"]["memory"] = 1 << 62
    snap = make(snap_doc)
    snap.compile(wls)
    snap.run_compiled()
    b1 = snap.last_results()
    admitted, deltas = snap.admit(snap.last_assignments())
    snap.run_compiled()
    b2 = snap.last_results()
    snap.close()
    ops = [{"op": "find", "podSets": w} for w in wls]
    admit_idx = [i for i, w in enumerate(wls) if all(not r["reason"] for r in b1[i])]
    ops += [{"op": "admit", "usage": synth.usage_records(wls[i], b1[i])} for i in admit_idx]
    ops += [{"op": "find", "podSets": w} for w in wls]
    res = oracle_lib.session(snap_doc, ops)
    assert b1 == res[:n]
    want = dict(zip(admit_idx, res[n:n + len(admit_idx)]))
    got = {int(i): bool(a) for i, a in admitted.tolist()}
    assert {i: got[i] for i in want} == want
    assert all(not got[i] for i in range(n) if i not in want)
    assert any(want.values()) and not all(want.values())
    assert b2 == res[n + len(admit_idx):]


# serial: the one-wave in-order chain (admit_kernel, KUEUE_TAS_CFG_SERIAL_ADMIT);
# default: the windowed admit_window_kernel — the same decisions either way
@pytest.mark.parametrize("serial", [False, True])
@pytest.mark.parametrize("tiny", [False, True])
def test_emulated_admit_batch(emu_lib, tiny, serial):  # noqa: F811
    _admit_batch(lambda d: TASFlavorSnapshot(d, lib=emu_lib, serial_admit=serial), huge_memory=tiny)


@pytest.mark.gpu
@pytest.mark.parametrize("serial", [False, True])
@pytest.mark.parametrize("tiny", [False, True])
def test_admit_batch_on_gpu(tiny, serial):
    _admit_batch(lambda d: TASFlavorSnapshot(d, serial_admit=serial), n=256, shape=(2, 4, 8, 16), huge_memory=tiny)


@pytest.mark.parametrize("phases", ["1", "6"])
def test_emulated_admit_phases(emu_lib, phases):  # noqa: F811
    """admit_window_kernel in phases with the rejection sweeps on the grid
    between them (KTAS_ADMIT_PHASES, default 6) or all in one workgroup (1):
    the same decisions as the oracle session."""
    import os

    old = os.environ.get("KTAS_ADMIT_PHASES")
    os.environ["KTAS_ADMIT_PHASES"] = phases
    try:
        _admit_batch(lambda d: TASFlavorSnapshot(d, lib=emu_lib), n=384, shape=(2, 2, 4, 8))
    finally:
        if old is None:
            os.environ.pop("KTAS_ADMIT_PHASES")
        else:
            os.environ["KTAS_ADMIT_PHASES"] = old


@pytest.mark.gpu
def test_admit_8192_phases_match_serial_on_gpu():
    """The 8-GPU admission load (8 x 1,024 gathered C3 candidates): grid
    sweeps between window phases, one in-kernel phase and the one-wave chain
    agree bit for bit."""
    import os

    import numpy as np

    doc, wls = synth.config_c3(n_workloads=8192)
    out = []
    for phases, serial in (("6", False), ("1", False), ("6", True)):
        os.environ["KTAS_ADMIT_PHASES"] = phases
        try:
            snap = TASFlavorSnapshot(doc, serial_admit=serial)
        finally:
            os.environ.pop("KTAS_ADMIT_PHASES")
        snap.compile(wls)
        snap.run_compiled()
        admitted, deltas = snap.admit(snap.last_assignments())
        out.append((admitted.copy(), np.sort(deltas, order=["leaf", "col"])))
        snap.close()
    for o in out[1:]:
        assert (out[0][0] == o[0]).all()
        assert (out[0][1] == o[1]).all()
    assert 0 < int(out[0][0][:, 1].sum()) < len(wls)


@pytest.mark.gpu
def test_admit_window_matches_serial_c3_on_gpu():
    # the C3 bench batch (1,024 workloads, heavy leaf overlap: most are
    # rejected after an earlier admission): window and chain agree bit for bit
    import numpy as np

    doc, wls = synth.config_c3(n_workloads=1024)
    out = []
    for serial in (False, True):
        snap = TASFlavorSnapshot(doc, serial_admit=serial)
        snap.compile(wls)
        snap.run_compiled()
        admitted, deltas = snap.admit(snap.last_assignments())
        out.append((admitted.copy(), np.sort(deltas, order=["leaf", "col"])))
        snap.close()
    assert (out[0][0] == out[1][0]).all()
    assert (out[0][1] == out[1][1]).all()
    assert 0 < int(out[0][0][:, 1].sum()) < len(wls)


def test_emulated_admit_record_order_and_errors(emu_lib):  # noqa: F811
    """kueue_tas_host_admit groups the quads per workload in the host pool's
    static parts: any quad order gives the same decisions and deltas as the
    gathered order; a workload id or record out of range is an error."""
    import numpy as np

    snap_doc, wls = synth.config_c2(n_workloads=64, shape=(2, 2, 4, 8))

    def fresh():
        s = TASFlavorSnapshot(snap_doc, lib=emu_lib)
        s.compile(wls)
        s.run_compiled()
        return s

    s = fresh()
    q = np.asarray(s.last_assignments(), dtype=np.int32).reshape(-1, 4)
    a1, d1 = s.admit(q.ravel())
    s.close()
    assert len(q) > 64 and a1[:, 1].any() and not a1[:, 1].all()
    s = fresh()
    a2, d2 = s.admit(np.ascontiguousarray(q[::-1]).ravel())
    s.close()
    assert a1.tolist() == a2.tolist()
    assert np.array_equal(np.sort(d1, order=["leaf", "col"]), np.sort(d2, order=["leaf", "col"]))
    for field, value, msg in ((0, 10**6, "workload id out of range"), (2, 10**7, "record out of range")):
        bad = q.copy()
        bad[np.nonzero(bad[:, 1] >= 0)[0][len(q) // 3], field] = value
        s = fresh()
        with pytest.raises(RuntimeError, match=msg):
            s.admit(bad.ravel())
        s.close()
