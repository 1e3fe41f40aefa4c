"""Bounded phase-2 memory (tas_device.hip eval_chunk, scratch_bound): the
BestFit-side select's list scratch sized per evaluation by the candidates its
walk can reach, its copy-on-write overlay by its kind, and its slots run in
groups whose buffers fit a byte budget.  Results must not depend on any of
it: a tiny budget (one select launch per slot), lists capped below what a
walk needs (every overflow re-runs the chunk unbounded) and the unbounded
lists all agree with the oracle (the reference's findTopologyAssignment,
tas_flavor_snapshot.go:519-594, has no such limits)."""
import os
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(lib, env, seed, n, gen=None, want_groups=None):
    rng = random.Random(seed)
    groups = reruns = 0

    def run():
        nonlocal groups, reruns
        for _ in range(n):
            case = (gen or synth.random_case)(rng)
            snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
            got = snap.find_topology_assignments_for_flavor(case["podSets"])
            g, r = snap.select_groups()
            groups = max(groups, g)
            reruns = max(reruns, r)
            snap.close()
            assert got == oracle_lib.run_case(case)["results"]

    _with_env(env, run)
    if want_groups:
        assert groups >= want_groups


def _batch(lib, env, n=96, shape=(2, 2, 4, 64)):
    """A C2 batch on small nodes (about two pods each): BestFit walks spread
    over several racks, so their leaf-level lists run long."""
    doc, wls = synth.config_c2(n_workloads=n, shape=shape)
    for nd in doc["nodes"]:
        nd["allocatable"]["cpu"] = 80000

    def run():
        snap = TASFlavorSnapshot(doc, lib=lib) if lib else TASFlavorSnapshot(doc)
        got = snap.find_topology_assignments_for_workloads(wls)
        out = (got, snap.select_groups(), snap.device_bytes())
        snap.close()
        return out

    got, groups, nbytes = _with_env(env, run)
    want, _ = oracle_lib.eval_workloads(doc, wls, threads=4)
    assert got == want
    return groups, nbytes


def test_emulated_phase2_groups_and_overflow(emu_lib):  # noqa: F811
    _check(emu_lib, {"KTAS_PHASE2_BUDGET": "1"}, 71, 25)
    _check(emu_lib, {"KTAS_SCRATCH_TEST_CAP": "2"}, 72, 25)
    (g, _), _ = _batch(emu_lib, {"KTAS_PHASE2_BUDGET": "1"})
    assert g > 1
    _batch(emu_lib, {"KTAS_SCRATCH_TEST_CAP": "4"})
    # the re-run path itself (an overflow re-runs the chunk with unbounded lists)
    (g, r), _ = _batch(emu_lib, {"KTAS_SCRATCH_TEST_RERUN": "1"})
    assert r > 0


def test_emulated_phase2_bytes(emu_lib):  # noqa: F811
    """The bounded lists hold less than the unbounded ones on a batch whose
    requests sit above the leaf level."""
    _, bounded = _batch(emu_lib, {})
    _, full = _batch(emu_lib, {"KTAS_SCRATCH_FULL": "1"})
    assert bounded[1] < full[1]


@pytest.mark.gpu
def test_phase2_groups_and_overflow_on_gpu():
    _check(None, {"KTAS_PHASE2_BUDGET": "1"}, 73, 80)
    _check(None, {"KTAS_SCRATCH_TEST_CAP": "2"}, 74, 80)
    (g, _), _ = _batch(None, {"KTAS_PHASE2_BUDGET": "1"}, n=512, shape=(4, 8, 8, 64))
    assert g > 1
    _batch(None, {"KTAS_SCRATCH_TEST_CAP": "4"}, n=512, shape=(4, 8, 8, 64))
    (g, r), _ = _batch(None, {"KTAS_SCRATCH_TEST_RERUN": "1"}, n=512, shape=(4, 8, 8, 64))
    assert r > 0
