"""Batched preemption search (the TAS part of preemption's `minimal`,
pkg/scheduler/preemption/preemption.go:307-345, with workloadFits :614-625
reduced to FindTopologyAssignmentsForWorkload(...).Failure() == nil) against
the oracle's restatement, which removes the candidates from a real oracle
snapshot one by one (RemoveUsage -> updateTASUsage) where the device path
evaluates every prefix in one batch under removal overlays.  The reference's
tests hold no TAS-level golden for this loop (scheduler_tas_test.go exercises
it through the whole scheduler), so parity rests on the find goldens that pin
the evaluation and on the oracle session."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth


def preemption_case(rng, gen=None):
    """A snapshot; `setup` ops admitting small copies of the workload (1-3
    pods per PodSet) one after another until the preemptor (1-2x the
    workload's counts) no longer fits or 16 are in; the admitted copies are
    the preemption candidates in shuffled order, plus sometimes a candidate
    whose records name no leaf."""
    case = gen(rng) if gen else synth.random_case(rng, max_nodes=rng.choice([6, 12, 24]))
    ps = case["podSets"]
    pre = [dict(p, count=max(1, p.get("count", 1) * rng.choice([1, 2]))) for p in ps]
    setup, cands = [], []
    for _ in range(16):
        res = oracle_lib.session(case, setup + [{"op": "find", "podSets": pre}])[-1]
        if any(r["reason"] for r in res):
            break
        small = [dict(p, count=rng.randint(1, 3)) for p in ps]
        got = oracle_lib.session(case, setup + [{"op": "find", "podSets": small}])[-1]
        u = synth.usage_records(small, got)
        if not u or any(r["reason"] for r in got):
            break
        setup.append({"op": "add", "usage": u})
        cands.append(u)
    rng.shuffle(cands)
    if rng.random() < 0.2:
        cands.insert(rng.randrange(len(cands) + 1),
                     [{"values": ["no-such-domain"], "singlePodRequests": {"cpu": 1}, "count": 1}])
    return case, setup, pre, cands


def _check(seed, n, lib=None, gen=None):
    rng = random.Random(seed)
    searched = 0
    for i in range(n):
        case, setup, pre, cands = preemption_case(rng, gen)
        if not cands:
            continue
        want = oracle_lib.preemption_search(case, setup, pre, cands)
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        for op in setup:
            snap.add_usage(op["usage"])
        got = snap.preemption_search(pre, cands)
        got.pop("profileMs")
        assert got == want, (i, got, want)
        # the search leaves the snapshot as it was (removals are overlays)
        after = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert after == oracle_lib.session(case, setup + [{"op": "find", "podSets": case["podSets"]}])[-1], i
        searched += got["firstFit"] >= 0
    assert searched > 0


def test_oracle_preemption_restatement_basic():
    # a candidate set whose removal frees exactly what the preemptor needs
    rng = random.Random(5)
    hits = 0
    for _ in range(30):
        case, setup, pre, cands = preemption_case(rng)
        if not cands:
            continue
        r = oracle_lib.preemption_search(case, setup, pre, cands)
        assert len(r["prefixFits"]) == len(cands)
        if r["firstFit"] >= 0:
            hits += 1
            assert r["prefixFits"][r["firstFit"]] and not any(r["prefixFits"][: r["firstFit"]])
            assert sorted(r["targets"]) == sorted(set(r["targets"]))
            assert set(r["targets"]) <= set(range(r["firstFit"] + 1))
    assert hits > 0


def test_emulated_preemption_search(emu_lib):  # noqa: F811
    _check(71, 120, lib=emu_lib)


@pytest.mark.gpu
def test_preemption_search_on_gpu():
    _check(81, 300)


@pytest.mark.gpu
def test_preemption_search_arith_on_gpu():
    _check(82, 120, gen=synth.arith_stress_case)
