"""Required node affinity and nodeSelector validation (findTopologyAssignment,
tas_flavor_snapshot.go:879-897 and fillInCounts :1605-1610).

Pinned by the reference's own fixtures (tests/golden/tas_affinity.json,
transcribed from pkg/scheduler/scheduler_tas_test.go:2618-2711 by
tools/transcribe_affinity_goldens.py); beyond them the oracle restatement of
the vendored nodeaffinity / labels helpers (oracle/k8s_selectors.h) is the
checker for randomized affinity (every operator, matchFields, empty terms)
and for the validation failure strings.  The kernels run on the CPU SIMT
emulator here and on the MI355X in the `gpu` tests."""
import json
import os
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "tas_affinity.json")


def _cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def _check_golden(case, results):
    (ps,) = case["podSets"]
    (r,) = results
    assert r["name"] == ps["name"]
    assert r["assignment"] == ps["wantAssignment"]
    if ps["wantReasonPinned"]:
        assert r["reason"] == ps["wantReason"]
    else:  # the reference pins "not admitted"; the text is the oracle's derivation
        assert r["reason"] != "" and r["reason"] == ps["wantReason"]


def test_oracle_matches_affinity_goldens():
    for case in _cases():
        _check_golden(case, oracle_lib.run_case(case)["results"])


def _invalid_podset(base, affinity=None, selector=None):
    ps = dict(base, affinity=affinity, nodeSelector=selector)
    for k in ("wantAssignment", "wantReason", "wantReasonPinned"):
        ps.pop(k, None)
    return ps


def _terms(*terms):
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": list(terms)}}}


# Validation failures with their text derived by hand from the vendored Go
# (nodeaffinity.go:214-293, selector.go:185-225, field/errors.go:63-117,
# generated.pb.go:22060-22107); the oracle must produce exactly these.
KNOWN_REASONS = [
    (_terms({"matchExpressions": [{"key": "k", "operator": "Foo", "values": ["v"]}]}), None,
     "invalid affinity node selectors: &NodeSelector{NodeSelectorTerms:[]NodeSelectorTerm{NodeSelectorTerm{"
     "MatchExpressions:[]NodeSelectorRequirement{NodeSelectorRequirement{Key:k,Operator:Foo,Values:[v],},},"
     "MatchFields:[]NodeSelectorRequirement{},},},}, reason: nodeSelectorTerms[0].matchExpressions[0].operator: "
     "Unsupported value: \"Foo\": supported values: \"In\", \"NotIn\", \"Exists\", \"DoesNotExist\", \"Gt\", \"Lt\""),
    (_terms({"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["a", "b"]}]}), None,
     "invalid affinity node selectors: &NodeSelector{NodeSelectorTerms:[]NodeSelectorTerm{NodeSelectorTerm{"
     "MatchExpressions:[]NodeSelectorRequirement{},MatchFields:[]NodeSelectorRequirement{NodeSelectorRequirement{"
     "Key:metadata.name,Operator:In,Values:[a b],},},},},}, reason: nodeSelectorTerms[0].matchFields[0].values: "
     "Invalid value: [\"a\",\"b\"]: must have one element"),
    (None, {"ok": "v!"},
     "invalid node selectors: map[ok:v!], reason: values[0][ok]: Invalid value: \"v!\": a valid label must be an "
     "empty string or consist of alphanumeric characters, '-', '_' or '.', and must start and end with an "
     "alphanumeric character (e.g. 'MyValue',  or 'my_value',  or '12345', regex used for validation is "
     "'(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?')"),
]

MORE_INVALID = [
    (_terms({"matchExpressions": [{"key": "a/b/c", "operator": "In", "values": []},
                                  {"key": "n", "operator": "Gt", "values": ["x", "y"]}]},
            {"matchFields": [{"key": "metadata.name", "operator": "Exists"}]}), None),
    (_terms({"matchExpressions": [{"key": "k", "operator": "Exists", "values": ["<v>"]}]}), None),
    (_terms({"matchExpressions": [{"key": "UPPER.io/" + "x" * 70, "operator": "DoesNotExist"}]}), None),
    (_terms({}, {"matchExpressions": [{"key": "/x", "operator": "NotIn", "values": ["y" * 64, "ok"]}]}), None),
    (None, {"-bad": "v!", "ok": "fine"}),
    (_terms({"matchExpressions": [{"key": "k", "operator": "In", "values": ["a"]}]}), {"a/b/c": "x"}),
]


def _run_reasons(snap_factory, case):
    base = case["podSets"][0]
    out = []
    for aff, sel, *_ in KNOWN_REASONS + [m + (None,) for m in MORE_INVALID]:
        ps = _invalid_podset(base, aff, sel)
        c = dict(case, podSets=[ps])
        want = oracle_lib.run_case(c)["results"]
        snap = snap_factory(c)
        got = snap.find_topology_assignments_for_flavor([ps])
        snap.close()
        out.append((got, want))
    return out


def test_oracle_known_validation_reasons():
    case = _cases()[0]
    for aff, sel, reason in KNOWN_REASONS:
        c = dict(case, podSets=[_invalid_podset(case["podSets"][0], aff, sel)])
        assert oracle_lib.run_case(c)["results"][0]["reason"] == reason


def test_emulated_validation_reasons_match_oracle(emu_lib):
    for got, want in _run_reasons(lambda c: TASFlavorSnapshot(c, lib=emu_lib), _cases()[0]):
        assert got == want


def test_emulated_affinity_goldens(emu_lib):
    for case in _cases():
        snap = TASFlavorSnapshot(case, lib=emu_lib)
        _check_golden(case, snap.find_topology_assignments_for_flavor(case["podSets"]))
        snap.close()


def _random_affinity_parity(seed, n, make_snap, max_nodes=60):
    rng = random.Random(seed)
    bad = []
    for i in range(n):
        case = synth.affinity_case(rng, max_nodes=max_nodes)
        want = oracle_lib.run_case(case)["results"]
        snap = make_snap(case)
        got = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        if got != want:
            bad.append((i, got, want))
            if len(bad) >= 3:
                break
    return bad


# split: the one-leaf staged fill with the ExclusionStats counted by fill_exclusion_kernel
@pytest.mark.parametrize("seed,split,max_nodes,n", [(61, False, 60, 200), (62, True, 60, 120), (63, False, 500, 40)])
def test_emulated_random_affinity_matches_oracle(emu_lib, seed, split, max_nodes, n):
    bad = _random_affinity_parity(seed, n, lambda c: TASFlavorSnapshot(c, lib=emu_lib, split_stats=split, pair_fill=not split),
                                  max_nodes=max_nodes)
    assert not bad, bad[0]


@pytest.mark.gpu
def test_affinity_goldens_on_gpu():
    for case in _cases():
        snap = TASFlavorSnapshot(case)
        _check_golden(case, snap.find_topology_assignments_for_flavor(case["podSets"]))
        snap.close()


@pytest.mark.gpu
def test_validation_reasons_on_gpu():
    for got, want in _run_reasons(lambda c: TASFlavorSnapshot(c), _cases()[0]):
        assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed,split,max_nodes,n", [(71, False, 60, 400), (72, True, 60, 200), (73, False, 600, 60)])
def test_random_affinity_on_gpu(seed, split, max_nodes, n):
    bad = _random_affinity_parity(seed, n, lambda c: TASFlavorSnapshot(c, split_stats=split, pair_fill=not split),
                                  max_nodes=max_nodes)
    assert not bad, bad[0]
