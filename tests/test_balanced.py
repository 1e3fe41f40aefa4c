"""TASBalancedPlacement (Alpha gate; tas_flavor_snapshot.go:906-917,
pkg/cache/scheduler/tas_balanced_placement.go) through the host layer: the
device computes phase 1 (fillInCounts + roll-up), kueue_tas_last_counters
hands the counters to the host algorithm (kueue_oss_amd/csrc/tas_balanced.h).

Pinned by the reference's 18 TestFindTopologyAssignments cases under the gate
(tas_cache_test.go:2437-3884, in tests/golden: every golden test runs them)
and, on seeded random cases, bit-exact against the oracle's restatement
(oracle/tas_oracle.cpp).  Where Go iterates a map (domainsPerLevel,
domain.children) both use lexicographic levelValues order; the random
generator does not avoid such ties, so those cases check the documented rule."""
import random

import pytest

import oracle_lib
from golden_util import diff_against_golden, load_cases
from kueue_oss_amd import TASFlavorSnapshot, synth

BALANCED = [c for c in load_cases() if c.get("featureGates", {}).get("TASBalancedPlacement")]


def test_goldens_cover_the_gate():
    assert len(BALANCED) == 18


def _random(make, seed, n, max_nodes):
    rng = random.Random(seed)
    changed = 0
    for i in range(n):
        case = synth.balanced_case(rng, max_nodes=max_nodes)
        want = oracle_lib.run_case(case)["results"]
        snap = make(case)
        got = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert got == want, (i, got, want)
        off = dict(case, featureGates=dict(case["featureGates"], TASBalancedPlacement=False))
        changed += oracle_lib.run_case(off)["results"] != want
    assert changed > n // 20  # the balanced branch decided a share of the cases


@pytest.mark.parametrize("list_cap", [0, 64])
def test_emulated_balanced_goldens(emu_lib, list_cap):
    for case in BALANCED:
        snap = TASFlavorSnapshot(case, list_cap=list_cap, lib=emu_lib)
        res = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert diff_against_golden(case, res) == [], case["line"]


@pytest.mark.parametrize("seed,max_nodes,n", [(1, 60, 150), (2, 200, 80)])
def test_emulated_balanced_random(emu_lib, seed, max_nodes, n):
    _random(lambda d: TASFlavorSnapshot(d, lib=emu_lib), seed, n, max_nodes)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,max_nodes,n", [(3, 60, 400), (4, 300, 200)])
def test_balanced_random_on_gpu(seed, max_nodes, n):
    _random(lambda d: TASFlavorSnapshot(d), seed, n, max_nodes)


@pytest.mark.gpu
def test_balanced_batch_on_gpu():
    # a nominate batch under the gate: balanced groups ride in the device
    # batch, their counters come back in a second batch of just those requests
    doc, wls = synth.config_c2(n_workloads=64, shape=(2, 4, 16, 16))
    doc = dict(doc, featureGates={"TASBalancedPlacement": True})
    want, _ = oracle_lib.eval_workloads(doc, wls)
    snap = TASFlavorSnapshot(doc)
    got = snap.find_topology_assignments_for_workloads(wls)
    snap.close()
    assert got == want
