"""v1beta2 compact TopologyAssignment encoding (pkg/util/tas/tas_assignment.go
:135-259): the oracle's restatement against the reference's own vectors
(tas_assignment_test.go bothWaysTestCases / oneWayTestCases, transcribed by
tools/extract_encoding_goldens.py)."""
import json
import os
import random

import pytest

import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "tas_v1beta2_encoding.json")))["cases"]


def test_fixture_inventory():
    assert len(CASES) == 12 and sum(c["bothWays"] for c in CASES) == 10


@pytest.mark.parametrize("case", [c for c in CASES if c["bothWays"]], ids=lambda c: f"L{c['line']}")
def test_oracle_v1beta2_from(case):
    assert oracle_lib.v1beta2_from(case["internal"]) == case["v1beta2"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"L{c['line']}")
def test_oracle_internal_from(case):
    got = oracle_lib.internal_from(case["v1beta2"])
    assert got == case["internal"]
    assert [d["count"] for d in got["domains"]] == case["podCounts"]
    assert len(got["domains"]) == case["totalDomainCount"]


# ---- the device encoder (explicit strings) and the host decoder ----
from kueue_oss_amd import TASFlavorSnapshot, synth  # noqa: E402

_TINY = {"name": "enc", "levels": ["kubernetes.io/hostname"],
         "nodes": [{"name": "n0", "labels": {"kubernetes.io/hostname": "n0"}, "allocatable": {"cpu": 1},
                    "taints": [], "unschedulable": False, "conditions": [{"type": "Ready", "status": "True"}]}],
         "pods": [], "tasUsage": [], "nodeLabels": {}, "flavorTolerations": [], "featureGates": {}}


def _check_encoder(snap, seed, n):
    both = [c for c in CASES if c["bothWays"]]
    assert snap.v1beta2_from([c["internal"] for c in both] + [None]) == [c["v1beta2"] for c in both] + [None]
    assert snap.internal_from([c["v1beta2"] for c in CASES]) == [c["internal"] for c in CASES]
    rng = random.Random(seed)
    tas = [synth.random_internal_assignment(rng) for _ in range(n)]
    want = [oracle_lib.v1beta2_from(t) if t is not None else None for t in tas]
    assert snap.v1beta2_from(tas) == want
    assert snap.internal_from(want) == [t if t is not None else None for t in tas]


def test_emulated_encoder_goldens_and_random(emu_lib):  # noqa: F811
    snap = TASFlavorSnapshot(_TINY, lib=emu_lib)
    _check_encoder(snap, 71, 150)
    snap.close()


@pytest.mark.gpu
def test_encoder_goldens_and_random_on_gpu():
    snap = TASFlavorSnapshot(_TINY)
    _check_encoder(snap, 72, 2000)
    snap.close()


def _find_v1beta2_parity(gen, seed, n, lib=None):
    rng = random.Random(seed)
    for i in range(n):
        case = gen(rng)
        want = oracle_lib.run_case(case)["results"]
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        got = snap.find_topology_assignments_v1beta2(case["podSets"])
        snap.close()
        exp = [{"name": r["name"], "topologyAssignment": oracle_lib.v1beta2_from(r["assignment"])
                if r["assignment"] is not None else None, "reason": r["reason"]} for r in want]
        assert got == exp, (i, got, exp)


def test_emulated_find_v1beta2(emu_lib):  # noqa: F811
    _find_v1beta2_parity(synth.random_case, 73, 80, lib=emu_lib)


@pytest.mark.gpu
def test_find_v1beta2_on_gpu():
    _find_v1beta2_parity(synth.random_case, 74, 300)
