"""Batched partial-admission search: PodSetReducer.Search
(pkg/scheduler/flavorassigner/podset_reducer.go:37-86, driven by
Scheduler.getInitialAssignments, pkg/scheduler/scheduler.go:720-739) over the
TAS fit of a workload, against the oracle's restatement
(oracle/tas_oracle.cpp podset_reducer_search, session op "partialAdmission"),
which walks sort.Search one probe at a time on an oracle snapshot.  The
device path evaluates sort.Search's decision tree speculatively, a batch of
levels per launch; the answer and the probe count must be the reference's
for any fits predicate (the tests use small batches too, so a search spans
many launches).  The reference's tests exercise the reducer only through the
whole scheduler (scheduler_test.go partial admission cases, quota-driven), so
no TAS-level golden exists: parity rests on the find goldens that pin every
evaluation and on the restatement below."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth


def reducer_case(rng, gen=None):
    """A snapshot whose workload is scaled up 2-8x (so its full counts often
    do not fit), each PodSet with a minCount, sometimes a PodSet outside TAS
    (count arithmetic only) and sometimes no room to reduce at all."""
    case = (gen or synth.random_case)(rng)
    ps = []
    for p in case["podSets"]:
        full = max(1, p.get("count", 1)) * rng.choice([1, 2, 4, 8])
        q = dict(p, count=full)
        r = rng.random()
        if r < 0.15:
            q["minCount"] = full  # no delta on this PodSet
        elif r < 0.3:
            pass  # minCount absent: Deref(MinCount, Count)
        else:
            q["minCount"] = rng.randint(0 if rng.random() < 0.2 else 1, full)
        ps.append(q)
    if rng.random() < 0.25:
        extra = dict(ps[0], name="quota-only", tas=False, podSetGroupName=None)
        extra["count"] = rng.randint(1, 40)
        extra["minCount"] = rng.randint(0, extra["count"])
        ps.insert(rng.randrange(len(ps) + 1), extra)
    return case, ps


def python_search(case, podsets, simulate_empty=False):
    """sort.Search over oracle sessions, a pure-Python restatement of
    podset_reducer.go:55-86 that checks the oracle's C++ one."""
    full = [p["count"] for p in podsets]
    deltas = [p["count"] - (p["minCount"] if p.get("minCount") is not None else p["count"]) for p in podsets]
    total = sum(deltas)
    if total == 0:
        return {"found": False, "counts": None, "results": None, "probes": 0}

    def fill(up):  # int32(int64(v) * int64(up) / int64(total)): Go truncates toward zero
        out = []
        for f, d in zip(full, deltas):
            num = d * up
            q = abs(num) // total
            out.append(f - (q if num >= 0 else -q))
        return out

    last_good, last_r, probes = 0, None, 0
    i, j = 0, total + 1
    while i < j:
        h = (i + j) >> 1
        cur = fill(h)
        reqs = [dict(p, count=c) for p, c in zip(podsets, cur) if p.get("tas", True) and c != 0]
        probes += 1
        rs = oracle_lib.session(case, [{"op": "find", "podSets": reqs, "simulateEmpty": simulate_empty}])[0] \
            if reqs else []
        f = all(not r["reason"] for r in rs)
        if f:
            last_good, last_r = h, rs
            j = h
        else:
            i = h + 1
    found = i == last_good
    return {"found": found, "counts": fill(last_good) if found else None, "results": last_r if found else None,
            "probes": probes}


def oracle_search(case, podsets, simulate_empty=False):
    return oracle_lib.session(case, [{"op": "partialAdmission", "podSets": podsets,
                                      "simulateEmpty": simulate_empty}])[0]


def test_oracle_reducer_restatement():
    rng = random.Random(17)
    found = lost = 0
    for _ in range(60):
        case, ps = reducer_case(rng)
        want = python_search(case, ps)
        got = oracle_search(case, ps)
        assert got == want
        if got["found"]:
            found += 1
            for c, p in zip(got["counts"], ps):
                lo = p["minCount"] if p.get("minCount") is not None else p["count"]
                assert lo <= c <= p["count"]
        elif got["probes"]:
            lost += 1
    assert found > 5 and lost > 0


def _check(seed, n, lib=None, gen=None, batches=(0, 1, 3, 7)):
    rng = random.Random(seed)
    searched = 0
    for i in range(n):
        case, ps = reducer_case(rng, gen)
        sim = rng.random() < 0.15
        want = oracle_search(case, ps, sim)
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        for mb in batches:
            got = snap.partial_admission_search(ps, simulate_empty=sim, max_batch=mb)
            for k in ("evaluations", "batches", "profileMs"):
                got.pop(k)
            assert got == want, (i, mb, got, want)
        # the search leaves the snapshot as it was
        after = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert after == oracle_lib.run_case(case)["results"], i
        searched += want["found"]
    assert searched > 0


def test_emulated_partial_admission_search(emu_lib):  # noqa: F811
    _check(91, 40, lib=emu_lib)


def test_emulated_partial_admission_batches(emu_lib):  # noqa: F811
    """A large totalDelta: the default batch (1,023 probes, ten levels) needs
    two launches, a batch of one probe needs one launch per level."""
    case = synth.random_case(random.Random(5), max_nodes=24)
    ps = [dict(p, count=max(1, p.get("count", 1)) * 3000, minCount=1) for p in case["podSets"]]
    want = oracle_search(case, ps)
    assert want["probes"] >= 11
    snap = TASFlavorSnapshot(case, lib=emu_lib)
    for mb in (0, 1):
        got = snap.partial_admission_search(ps, max_batch=mb)
        assert {k: got[k] for k in want} == want
        if mb == 0:
            assert 2 <= got["batches"] <= (want["probes"] + 9) // 10
        else:
            assert got["batches"] <= want["probes"]
    snap.close()


@pytest.mark.gpu
def test_partial_admission_search_on_gpu():
    _check(92, 200)


@pytest.mark.gpu
def test_partial_admission_search_arith_on_gpu():
    _check(93, 80, gen=synth.arith_stress_case, batches=(0, 2))
