"""fill_pair_kernel: the staged fill with two adjacent leaves per thread
(fillInCounts tas_flavor_snapshot.go:1568-1647 + the fused first level of
fillInCountsHelper :1658-1719), ExclusionStats counted in its class loop.
Checked bit-exactly against the oracle for single-run and multi-run chunks,
fused fan-outs 2 / 4 / 8 / 16 / 32 / 64, no fused parents (fan-out > 64, odd
leaf counts: the partial last group), leader groups, taints, selectors and
affinity; the one-leaf staged kernel (KUEUE_TAS_CFG_NO_PAIR_FILL) must give
the same results (that run also takes the KUEUE_TAS_CFG_FUSED_TOP roll-up:
rollup_top_kernel).  kueue_tas_last_fill_paths pins which kernel ran."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

PAIR = 8192


def _batch(make, doc, wls):
    want, _ = oracle_lib.eval_workloads(doc, wls, threads=4)
    snap = make(doc)
    snap.compile(wls)
    snap.run_compiled(flags=TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES)
    got = snap.last_results()
    paths = snap.last_stats()["fill_paths"]
    snap.close()
    mism = [i for i in range(len(wls)) if got[i] != want[i]]
    assert mism == [], (mism[:5], got[mism[0]], want[mism[0]])
    return paths


def _configs(scale):
    """(name, doc, workloads) covering the pair kernel's variants."""
    n = 64 * scale
    yield "c3 fan-out 32", *synth.config_c3(seed=3, n_workloads=3 * n, shape=(2, 2, 4 * scale, 32))
    yield "c3 fan-out 64", *synth.config_c3(seed=4, n_workloads=n, shape=(2, 2, 2 * scale, 64))
    yield "c3 fan-out 16", *synth.config_c3(seed=5, n_workloads=n, shape=(2, 2, 4 * scale, 16))
    yield "c3 fan-out 4", *synth.config_c3(seed=6, n_workloads=n, shape=(2, 4, 8 * scale, 4))
    yield "c3 fan-out 8", *synth.config_c3(seed=10, n_workloads=n, shape=(2, 4, 4 * scale, 8))
    yield "c3 fan-out 101 (no fused parents, odd N)", *synth.config_c3(seed=7, n_workloads=n, shape=(1, 1, 3, 101))
    yield "c2 mixed", *synth.config_c2(seed=8, n_workloads=n, shape=(2, 2, 4 * scale, 32))
    yield "c4 leaders", *synth.config_c4(seed=9, n_workloads=8 * scale, shape=(2, 2, 4 * scale, 16))


def _run(make_pair, make_staged, scale):
    for name, doc, wls in _configs(scale):
        paths = _batch(make_pair, doc, wls)
        assert paths & PAIR, name
        assert _batch(make_staged, doc, wls) & PAIR == 0, name
    # fan-out 2: one parent per lane (the smallest fused fan-out the kernel takes)
    doc, wls = synth.config_c3(seed=11, n_workloads=64 * scale, shape=(2, 4, 16 * scale, 2))
    assert _batch(make_pair, doc, wls) & PAIR


def _random(make, seed, n):
    rng = random.Random(seed)
    paths = 0
    for _ in range(n):
        case = synth.random_case(rng)
        snap = make(case)
        snap.compile([case["podSets"]])
        snap.run_compiled()
        got = snap.last_results()[0]
        paths |= snap.last_stats()["fill_paths"]
        snap.close()
        assert got == oracle_lib.run_case(case)["results"]
    return paths


def test_emulated_pair_fill(emu_lib):  # noqa: F811
    _run(lambda d: TASFlavorSnapshot(d, lib=emu_lib), lambda d: TASFlavorSnapshot(d, lib=emu_lib, pair_fill=False, fused_top=True), 1)
    assert _random(lambda d: TASFlavorSnapshot(d, lib=emu_lib), 31, 40) & PAIR


@pytest.mark.gpu
def test_pair_fill_on_gpu():
    _run(lambda d: TASFlavorSnapshot(d), lambda d: TASFlavorSnapshot(d, pair_fill=False, fused_top=True), 4)
    assert _random(lambda d: TASFlavorSnapshot(d), 32, 150) & PAIR
