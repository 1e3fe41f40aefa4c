"""The staged fill's fused roll-up of ragged leaf parents:
parents of 1..64 leaves packed whole into wave slots (DevSnap::wave_tab),
segmented DPP scans, the segment's last lane writing the parent's
fillInCountsHelper values (tas_flavor_snapshot.go:1658-1719) and its
positive-child mask; without leader classes, fill_pair_kernel's ragged mode
(two leaves per lane, parents of 1..128 leaves in 128-leaf slots,
DevSnap::wave_tab2: segmented scans over the lanes' pair summaries, no
positive-child masks when a parent is wider than 64).  Checked bit-exactly
against the oracle on ragged C3J-style snapshots and random trees; parents
of more than 128 leaves take the unfused roll-up (the same results).
kueue_tas_last_fill_paths pins which path ran."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

RAGGED, UNIFORM, RAGGED_PAIR = 2048, 4096, 32768


def _batch(make, doc, wls):
    want, _ = oracle_lib.eval_workloads(doc, wls, threads=4)
    snap = make(doc)
    snap.compile(wls)
    snap.run_compiled()
    got = snap.last_results()
    paths = snap.last_stats()["fill_paths"]
    snap.close()
    mism = [i for i in range(len(wls)) if got[i] != want[i]]
    assert mism == [], (mism[:5], got[mism[0]], want[mism[0]])
    return paths


def _c3j(make, shape, rack_sizes, n):
    doc, wls = synth.config_c3j(seed=sum(shape) + rack_sizes[1], n_workloads=n, shape=shape, rack_sizes=rack_sizes)
    return _batch(make, doc, wls)


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


def test_emulated_ragged_rollup(emu_lib):  # noqa: F811
    make = lambda d: TASFlavorSnapshot(d, lib=emu_lib)  # noqa: E731
    assert _c3j(make, (2, 2, 3), (1, 64), 24) & RAGGED_PAIR
    assert _c3j(make, (1, 2, 2), (60, 80), 12) & RAGGED_PAIR  # parents of > 64 leaves: no masks
    assert _c3j(make, (1, 1, 2), (120, 140), 8) & (RAGGED | UNIFORM) == 0  # a parent of > 128 leaves
    assert _random(make, 17, 40) & RAGGED
    # the one-leaf staged kernel's ragged mode (the pair kernel switched off)
    make1 = lambda d: TASFlavorSnapshot(d, lib=emu_lib, pair_fill=False)  # noqa: E731
    assert _c3j(make1, (2, 2, 3), (1, 64), 24) & RAGGED
    assert not _c3j(make1, (2, 2, 3), (1, 64), 24) & RAGGED_PAIR


@pytest.mark.gpu
def test_ragged_rollup_on_gpu():
    make = lambda d: TASFlavorSnapshot(d)  # noqa: E731
    assert _c3j(make, (2, 4, 16), (1, 64), 256) & RAGGED_PAIR
    assert _c3j(make, (2, 4, 16), (20, 44), 256) & RAGGED_PAIR
    assert _c3j(make, (1, 4, 8), (50, 90), 96) & RAGGED_PAIR
    assert _c3j(make, (1, 2, 4), (100, 128), 64) & RAGGED_PAIR
    assert _c3j(make, (1, 2, 4), (120, 200), 64) & (RAGGED | UNIFORM) == 0
    assert _random(make, 18, 150) & RAGGED
    make1 = lambda d: TASFlavorSnapshot(d, pair_fill=False)  # noqa: E731
    assert _c3j(make1, (2, 4, 16), (20, 44), 256) & RAGGED
