"""fill_pair_kernel: the staged fill with two adjacent leaves per thread
(fillInCounts tas_flavor_snapshot.go:1568-1647 + the fused first level of
fillInCountsHelper :1658-1719), ExclusionStats counted in its class loop.
Checked bit-exactly against the oracle for single-run and multi-run chunks
(C3J-like: a request signature per workload over ragged racks),
fused fan-outs 2 / 4 / 8 / 16 / 32 / 64, no fused parents (fan-out > 64, odd
leaf counts: the partial last group), leader groups, taints, selectors and
affinity; the one-leaf staged kernel (KUEUE_TAS_CFG_NO_PAIR_FILL) must give
the same results (that run also takes the KUEUE_TAS_CFG_FUSED_TOP roll-up:
rollup_top_kernel), and so must the pair kernel's per-leaf classification
(KUEUE_TAS_CFG_NO_CATEGORY_FILL) beside its default leaf categories: waves
with more than 64 categories (a label of many values) fall back to it, and
leaves out of the snapshot (nodes gone NotReady) form a category of their
own.  kueue_tas_last_fill_paths pins which kernel ran."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

PAIR = 8192
CATEGORY = 65536
LFC_FILL = 131072  # the fast-LFC chunk tables accumulated by the fill (no lfc_hist_kernel)


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
    # enough workloads per request signature for single-run chunks (>= 8 classes: the leaf categories)
    yield "c3 fan-out 32", *synth.config_c3(seed=3, n_workloads=6 * n, shape=(2, 2, 4 * scale, 32))
    yield "c3 fan-out 64", *synth.config_c3(seed=4, n_workloads=n, shape=(2, 2, 2 * scale, 64))
    yield "c3 fan-out 16", *synth.config_c3(seed=5, n_workloads=n, shape=(2, 2, 4 * scale, 16))
    yield "c3 fan-out 4", *synth.config_c3(seed=6, n_workloads=n, shape=(2, 4, 8 * scale, 4))
    yield "c3 fan-out 8", *synth.config_c3(seed=10, n_workloads=n, shape=(2, 4, 4 * scale, 8))
    yield "c3 fan-out 101 (no fused parents, odd N)", *synth.config_c3(seed=7, n_workloads=n, shape=(1, 1, 3, 101))
    yield "c2 mixed", *synth.config_c2(seed=8, n_workloads=n, shape=(2, 2, 4 * scale, 32))
    yield "c4 leaders", *synth.config_c4(seed=9, n_workloads=8 * scale, shape=(2, 2, 4 * scale, 16))
    # every workload its own request signature (multi-run chunks) over ragged
    # racks, full GPU leaves excluded by resource
    yield "c3j multi-run", *synth.config_c3j(seed=13, n_workloads=2 * n, shape=(2, 2, 4 * scale))


def _run(make_pair, make_staged, scale, make_percls=None, make_lfc=None):
    for name, doc, wls in _configs(scale):
        paths = _batch(make_pair, doc, wls)
        assert paths & PAIR, name
        assert paths & CATEGORY or name != "c3 fan-out 32", name
        assert paths & LFC_FILL == 0, name  # lfc_hist_kernel by default
        if make_lfc is not None:
            assert _batch(make_lfc, doc, wls) & LFC_FILL or name != "c3 fan-out 32", name
        assert _batch(make_staged, doc, wls) & (PAIR | CATEGORY) == 0, name
        if make_percls is not None:
            assert _batch(make_percls, doc, wls) & (PAIR | CATEGORY) == PAIR, name
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


def _many_categories(make, scale):
    """Leaf categories beyond one wave's 64 (a label with a value per leaf of a
    128-leaf wave: the per-leaf fallback), and leaves gone out of the
    snapshot (dead-leaf category) between loads."""
    import copy

    doc, wls = synth.config_c3(seed=12, n_workloads=384 * scale, shape=(2, 2, 4 * scale, 32))
    # a staged label column (sorts first) of many values in the first half of
    # the leaves, selected by a quarter of the workloads: those blocks'
    # categories overflow the table
    for i, nd in enumerate(doc["nodes"]):
        nd["labels"]["a.example.com/slot"] = f"s{i % 97 if i < len(doc['nodes']) // 2 else i % 3}"
    for k, w in enumerate(wls):
        if k % 4 == 1:
            w[0]["nodeSelector"] = dict(w[0].get("nodeSelector") or {}, **{"a.example.com/slot": f"s{k % 3}"})
    gone = [copy.deepcopy(doc["nodes"][k]) for k in range(5, len(doc["nodes"]), 37)]
    for nd in gone:
        nd["conditions"] = [{"type": "Ready", "status": "False"}]
    names = {nd["name"] for nd in gone}
    doc_after = dict(doc, nodes=[next((g for g in gone if g["name"] == nd["name"]), nd) if nd["name"] in names else nd
                                 for nd in doc["nodes"]])
    want, _ = oracle_lib.eval_workloads(doc_after, wls, threads=4)
    snap = make(doc)
    snap.compile(wls)
    assert not snap.update_nodes(gone)  # in place: the leaves leave the device snapshot
    snap.run_compiled(flags=TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES)
    got = snap.last_results()
    paths = snap.last_stats()["fill_paths"]
    snap.close()
    mism = [i for i in range(len(wls)) if got[i] != want[i]]
    assert mism == [], (mism[:5], got[mism[0]], want[mism[0]])
    return paths


def test_emulated_pair_fill(emu_lib):  # noqa: F811
    _run(lambda d: TASFlavorSnapshot(d, lib=emu_lib), lambda d: TASFlavorSnapshot(d, lib=emu_lib, pair_fill=False, fused_top=True), 1,
         lambda d: TASFlavorSnapshot(d, lib=emu_lib, category_fill=False),
         lambda d: TASFlavorSnapshot(d, lib=emu_lib, lfc_in_fill=True))
    assert _random(lambda d: TASFlavorSnapshot(d, lib=emu_lib), 31, 40) & PAIR
    # lean and per-leaf blocks of one launch accumulate the LFC tables together
    assert _many_categories(lambda d: TASFlavorSnapshot(d, lib=emu_lib, lfc_in_fill=True), 1) \
        & (CATEGORY | LFC_FILL) == CATEGORY | LFC_FILL


@pytest.mark.gpu
def test_pair_fill_on_gpu():
    _run(lambda d: TASFlavorSnapshot(d), lambda d: TASFlavorSnapshot(d, pair_fill=False, fused_top=True), 4,
         lambda d: TASFlavorSnapshot(d, category_fill=False), lambda d: TASFlavorSnapshot(d, lfc_in_fill=True))
    assert _random(lambda d: TASFlavorSnapshot(d), 32, 150) & PAIR
    assert _random(lambda d: TASFlavorSnapshot(d, lfc_in_fill=True), 33, 100) & PAIR
    assert _many_categories(lambda d: TASFlavorSnapshot(d, lfc_in_fill=True), 4) & (CATEGORY | LFC_FILL) == CATEGORY | LFC_FILL
