"""The staged fill's fused roll-up of ragged leaf parents:
parents of 1..64 leaves packed whole into wave slots (DevSnap::wave_tab),
segmented DPP scans, the segment's last lane writing the parent's
fillInCountsHelper values (tas_flavor_snapshot.go:1658-1719) and its
positive-child mask; without leader classes, fill_pair_kernel's ragged mode
(two leaves per lane, parents of 1..128 leaves in 128-leaf slots,
DevSnap::wave_tab2: segmented scans over the lanes' pair summaries, no
positive-child masks when a parent is wider than 64; a parent wider than 128
leaves in 128-leaf pieces of its own whose sums add atomically into the
zeroed parent, its sliceState at the slice level finished after the fill).
Checked bit-exactly against the oracle on ragged C3J-style snapshots, random
trees, a C3 variant with 256-node racks and a block -> hostname topology of
1,024-node blocks; with leader classes parents wider than 64 take the
unfused roll-up (the same results).  kueue_tas_last_fill_paths pins which
path ran."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

RAGGED, UNIFORM, RAGGED_PAIR = 2048, 4096, 32768


def _batch(make, doc, wls):
    want, _ = oracle_lib.eval_workloads(doc, wls, threads=16 if len(doc["nodes"]) > 50000 else 4)
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


def _wide_sliced(make, n):
    """Workloads sliced at the leaves' parent level (podSetSliceRequiredTopology
    rack, slice size 4) over racks wider than a fill slot: the wide parents'
    sliceState = state / sliceSize after the pieces are summed."""
    doc, wls = synth.config_c3j(seed=5, n_workloads=n, shape=(1, 2, 3), rack_sizes=(100, 300))
    for k, w in enumerate(wls):
        tr = w[0].get("topologyRequest") or {}
        if k % 2 == 0:
            w[0]["topologyRequest"] = dict(tr, required=synth.BLOCK, preferred=None, unconstrained=None,
                                           podSetSliceRequiredTopology=synth.RACK, podSetSliceSize=4)
            w[0]["count"] = 4 * max(1, w[0]["count"] // 4)
    return _batch(make, doc, wls)


def _block_host(n):
    """C3 reshaped to a block -> hostname topology: 128 blocks of 1,024 nodes
    (the leaves' parents far wider than a fill slot); rack requests become
    block requests."""
    doc, wls = synth.config_c3(n_workloads=n, shape=(1, 128, 32, 32))
    doc = dict(doc, levels=[synth.BLOCK, synth.HOST])
    for w in wls:
        tr = w[0].get("topologyRequest")
        if tr:
            for k in ("required", "preferred"):
                if tr.get(k) == synth.RACK:
                    tr[k] = synth.BLOCK
    return doc, wls


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
    assert _c3j(make, (1, 1, 2), (120, 140), 8) & RAGGED_PAIR  # a parent of > 128 leaves: pieces
    assert _c3j(make, (1, 1, 3), (150, 400), 12) & RAGGED_PAIR  # several wide parents beside narrow ones
    assert _wide_sliced(make, 4) & RAGGED_PAIR
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
    assert _c3j(make, (1, 2, 4), (120, 200), 64) & RAGGED_PAIR
    assert _c3j(make, (1, 2, 4), (300, 1100), 64) & RAGGED_PAIR
    assert _wide_sliced(make, 16) & RAGGED_PAIR
    assert _random(make, 18, 150) & RAGGED
    make1 = lambda d: TASFlavorSnapshot(d, pair_fill=False)  # noqa: E731
    assert _c3j(make1, (2, 4, 16), (20, 44), 256) & RAGGED


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_wide_parents_full_size_on_gpu():
    """a 256-node-rack C3 (131,072 nodes) and a block ->
    hostname topology of 1,024-node blocks, fused in the fill (no unfused
    leaf-level roll-up), against the 16-thread oracle."""
    make = lambda d: TASFlavorSnapshot(d)  # noqa: E731
    doc, wls = synth.config_c3(n_workloads=512, shape=(4, 16, 8, 256))
    assert _batch(make, doc, wls) & RAGGED_PAIR
    doc, wls = _block_host(512)
    assert _batch(make, doc, wls) & RAGGED_PAIR
