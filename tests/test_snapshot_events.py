"""Device-resident snapshot maintenance: non-TAS pod
events applied to a built snapshot in place (nonTasUsageCache.update/delete,
pkg/cache/scheduler/tas_non_tas_pod_cache.go:46-116, folded into the leaves'
freeCapacity as TASFlavorCache.snapshot does, tas_flavor.go:124-137) must give
the same evaluations as the reference's per-cycle rebuild — the oracle built
from scratch with the events appended to the snapshot's pod list, which it
replays through the same cache semantics (a terminated pod is the cache's
delete)."""
import copy
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth
from test_emu_parity import emu_lib  # noqa: F401  (fixture)

GI = 1 << 30


def pod_events(rng, case, n):
    """Random pod events: new pods, replacements of known pods (node move,
    resize, new resource names), deletions, terminations, unknown nodes."""
    names = [nd["name"] for nd in case["nodes"]] or ["nowhere"]
    known = [(p["namespace"], p["name"]) for p in case.get("pods", [])]
    evs = []
    for k in range(n):
        r = rng.random()
        if known and r < 0.35:
            ns, name = rng.choice(known)
        else:
            ns, name = "ev", f"e{k}"
            known.append((ns, name))
        ev = {"namespace": ns, "name": name, "nodeName": rng.choice(names) if rng.random() < 0.95 else "ghost",
              "phase": rng.choice(["Running", "Running", "Running", "Pending", "Succeeded", "Failed"]), "requests": {}}
        for res in rng.sample(["cpu", "memory", "example.com/gpu", "example.com/new"], rng.randint(0, 3)):
            ev["requests"][res] = (rng.choice([0, 250, 1000, 4000]) if res == "cpu" else
                                   rng.choice([0, GI // 2, 2 * GI]) if res == "memory" else rng.choice([0, 1, 2]))
        if rng.random() < 0.15:
            ev["delete"] = True
        evs.append(ev)
    return evs


def _oracle_pods(evs):
    return [dict(e, phase="Succeeded") if e.get("delete") else e for e in evs]


def _check(seed, n, lib=None, gen=None):
    rng = random.Random(seed)
    for i in range(n):
        case = (gen or synth.random_case)(rng)
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        ref = copy.deepcopy(case)
        ref.setdefault("pods", [])
        for step in range(3):
            evs = pod_events(rng, ref, rng.randint(1, 8))
            snap.update_pods(evs)
            ref["pods"] += _oracle_pods(evs)
            got = snap.find_topology_assignments_for_flavor(case["podSets"])
            want = oracle_lib.run_case(ref)["results"]
            assert got == want, (i, step, evs, got, want)
        snap.close()


def test_emulated_pod_events(emu_lib):  # noqa: F811
    _check(91, 60, lib=emu_lib)


@pytest.mark.gpu
def test_pod_events_on_gpu():
    _check(92, 200)


@pytest.mark.gpu
def test_pod_events_arith_on_gpu():
    _check(93, 100, gen=synth.arith_stress_case)
