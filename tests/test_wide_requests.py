"""Phase-1 kernel variants the bench configs never reach, each
checked bit-exactly against the oracle on batches built to reach it
(synth.wide_case):

* batches whose requests span more than 8 resource columns: the generic
  ``fill_leaves_kernel<16>`` / ``<32>`` (up to 21 request terms);
* more than 32 taint profiles: the staged fill reading taint rows from
  global memory and ``fill_exclusion_kernel<false>``;
* more than 64 ExclusionStats slots (3 + taint strings + columns): global
  atomics instead of the LDS partials;
* nodes with 47 resource names (more than the 32 device columns): only
  requested resources become columns (FlavorSnapshot::wanted_columns);
* nodeSelectors of 9..12 pairs (``labels.ValidatedSelectorFromSet``,
  vendor/k8s.io/apimachinery/pkg/labels/selector.go:954-968, any size): the
  pairs beyond the 8 inline ones of kueue_tas_eval_req go through
  KUEUE_TAS_F_SELECTOR_EXT; selector columns beyond the four held in
  registers, required node affinity, leader groups and slices ride along.

Each test also pins (kueue_tas_last_fill_paths) that the batch really ran
the variant it is named after."""
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

STAGED, STAGED_GT, G4, G8, G16, G32 = 1, 2, 4, 8, 16, 32
STAGED_GL, GLOBAL_STATS, EXCL, EXCL_GT, SEL_EXT = 64, 128, 256, 512, 1024
PAIR = 8192

WANT = {
    "cols": (G16 | G32 | GLOBAL_STATS | SEL_EXT, 0),
    "profiles": (STAGED_GT | EXCL_GT | STAGED_GL | SEL_EXT, 0),
    "slots": (GLOBAL_STATS | SEL_EXT, STAGED | STAGED_GT),
    "manyres": (SEL_EXT, 0),  # (47 names: only the requested ones become columns, no refusal)
}
# the same batches through fill_pair_kernel (two leaves per thread, stats in
# its loop: no fill_exclusion_kernel)
WANT_PAIR = {
    "profiles": (STAGED_GT | STAGED_GL | SEL_EXT | PAIR, 0),
    "slots": (GLOBAL_STATS | SEL_EXT | PAIR, STAGED | STAGED_GT),
}


def _run(make, variant, seeds, n_nodes, n_workloads, want_paths=None):
    paths = 0
    fits = fails = 0
    for seed in seeds:
        doc, wls = synth.wide_case(random.Random(seed), variant, n_nodes=n_nodes, n_workloads=n_workloads)
        want, _ = oracle_lib.eval_workloads(doc, wls)
        snap = make(doc)
        snap.compile(wls)
        snap.run_compiled()
        got = snap.last_results()
        paths |= snap.last_stats()["fill_paths"]
        snap.close()
        mism = [i for i in range(len(wls)) if got[i] != want[i]]
        assert mism == [], (variant, seed, mism[:5], got[mism[0]], want[mism[0]])
        fits += sum(1 for w in want for r in w if r["assignment"])
        fails += sum(1 for w in want for r in w if r["reason"])
    every, some = want_paths or WANT[variant]
    assert paths & every == every, (variant, hex(paths))
    assert some == 0 or paths & some, (variant, hex(paths))
    assert fits > 0 and fails > 0, (fits, fails)  # both outcomes (placements and ExclusionStats strings)


@pytest.mark.parametrize("variant", ["cols", "profiles", "slots", "manyres"])
def test_emulated_wide_variants(emu_lib, variant):
    _run(lambda d: TASFlavorSnapshot(d, lib=emu_lib, pair_fill=False, split_stats=True), variant, [0, 1], 300, 24)


@pytest.mark.parametrize("variant", ["profiles", "slots"])
def test_emulated_wide_variants_pair(emu_lib, variant):
    _run(lambda d: TASFlavorSnapshot(d, lib=emu_lib), variant, [0, 1], 1600, 24, WANT_PAIR[variant])  # racks > 64 leaves


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["cols", "profiles", "slots", "manyres"])
def test_wide_variants_on_gpu(variant):
    _run(lambda d: TASFlavorSnapshot(d, pair_fill=False, split_stats=True), variant, [0, 1, 2, 3], 2500, 96)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["profiles", "slots"])
def test_wide_variants_pair_on_gpu(variant):
    _run(lambda d: TASFlavorSnapshot(d), variant, [0, 1, 2, 3], 2560, 96, WANT_PAIR[variant])


@pytest.mark.gpu
def test_wide_variants_small_lds_on_gpu():
    # list_cap 64: the same batches through the lazy / global-sort / histogram walks
    _run(lambda d: TASFlavorSnapshot(d, list_cap=64), "cols", [5], 2500, 64, (GLOBAL_STATS | SEL_EXT, G16 | G32))
