"""Snapshot queries the scheduler's other callers make on a TAS snapshot
(kueue_tas.h "snapshot queries"), against the reference's own table tests
(tests/golden/snapshot_queries.json, written by
tools/transcribe_query_goldens.py):

  HasLevel                         tas_flavor_snapshot.go:1065  TestHasLevel :362-428
  ResourceQuantityString           requests.go:147              TestResourceQuantityRoundTrips requests_test.go:320-380
  SerializeFreeCapacityPerDomain   tas_flavor_snapshot.go:320   TestFreeCapacityPerDomain :33-72
  IsTopologyAssignmentStale        tas_flavor_snapshot.go:736   (no table test of its own: cases here
                                                                  follow its three lines, parity unpinned)

Run through the emulated build of the product library on CPU and the real
one on the GPU."""
import json
import os

import pytest

from kueue_oss_amd import TASFlavorSnapshot, native

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "snapshot_queries.json")))
HOST = "kubernetes.io/hostname"


def _node(name, labels, alloc):
    return {"name": name, "labels": labels, "allocatable": alloc, "taints": [], "unschedulable": False,
            "conditions": [{"type": "Ready", "status": "True"}]}


def _has_level(make):
    g = GOLD["has_level"]
    snap = make({"levels": g["levels"], "nodes": [_node("n", {"level-1": "a", "level-2": "b"}, {"cpu": 1})]})
    got = {c["name"]: snap.has_level(c["request"]) for c in g["cases"]}
    snap.close()
    assert got == {c["name"]: c["want"] for c in g["cases"]}


def _has_level_layers(make):
    # TASMultiLayerTopology: every additional layer's topology must resolve (:1079-1085)
    levels = ["l1", "l2", "l3"]
    nodes = [_node("n", {"l1": "a", "l2": "b", "l3": "c"}, {"cpu": 1})]
    req = {"required": "l1", "podsetSliceRequiredTopologyConstraints": [{"topology": "l2", "size": 2},
                                                                        {"topology": "nope", "size": 1}]}
    for gate, want in ((False, True), (True, False)):
        snap = make({"levels": levels, "nodes": nodes, "featureGates": {"TASMultiLayerTopology": gate}})
        assert snap.has_level(req) is want
        # the slice level key is the first constraint's topology
        assert snap.has_level({"required": "l1", "podsetSliceRequiredTopologyConstraints":
                               [{"topology": "zz", "size": 2}]}) is False
        snap.close()


def _free_capacity(make):
    g = GOLD["free_capacity"]
    nodes, usage = [], []
    for leaf, st in sorted(g["leaves"].items()):
        nodes.append(_node(leaf, {HOST: leaf}, st["freeCapacity"]))
        usage.append({"values": [leaf], "singlePodRequests": st["tasUsage"], "count": 1})
    snap = make({"levels": [HOST], "nodes": nodes, "tasUsage": usage})
    got = snap.serialize_free_capacity_per_domain()
    snap.close()
    # the golden is json.Marshal's text; this snapshot's tasUsage also holds
    # pods:1 per usage record (updateTASUsage adds pods:count, :257-260; the
    # reference test sets leafDomain.tasUsage directly)
    want = json.loads(g["expected"])
    assert json.dumps(want, sort_keys=True, separators=(",", ":")) == g["expected"]
    for d in want.values():
        d["tasUsage"]["pods"] = "1"
    assert got == json.dumps(want, sort_keys=True, separators=(",", ":"))


def _stale(make):
    levels = ["block", "rack", HOST]
    nodes = [_node(f"n{b}{r}{k}", {"block": f"b{b}", "rack": f"r{r}", HOST: f"n{b}{r}{k}"}, {"cpu": 1000})
             for b in range(2) for r in range(2) for k in range(2)]
    snap = make({"levels": levels, "nodes": nodes})

    def ta(lv, vals):
        return {"levels": lv, "domains": [{"values": v, "count": 1} for v in vals]}

    assert snap.is_topology_assignment_stale(ta([HOST], [["n000"], ["n111"]])) == (False, "")
    assert snap.is_topology_assignment_stale(ta([HOST], [["n000"], ["gone"], ["gone2"]])) == (True, "gone")
    assert snap.is_topology_assignment_stale(ta(["block", "rack"], [["b0", "r1"], ["b1", "r0"]])) == (False, "")
    assert snap.is_topology_assignment_stale(ta(["block", "rack"], [["b0", "r9"]])) == (True, "b0")
    assert snap.is_topology_assignment_stale(ta(["block"], [["b1"]])) == (False, "")
    assert snap.is_topology_assignment_stale(ta([HOST], [])) == (False, "")
    # a node that leaves the snapshot (NotReady) makes its assignment stale
    gone = dict(nodes[0], conditions=[{"type": "Ready", "status": "False"}])
    snap.update_nodes([gone])
    assert snap.is_topology_assignment_stale(ta([HOST], [["n001"], ["n000"]])) == (True, "n000")
    snap.close()


CHECKS = [_has_level, _has_level_layers, _free_capacity, _stale]


def test_quantity_strings_pinned():
    lib = native.load_library()  # no device call: the formatter is host code
    for res, v, want in GOLD["quantity"]["cases"]:
        assert native.resource_quantity_string(res, v, lib=lib) == want, (res, v)
    # edges of the same rules: zero, negatives, hugepages-*, other resources
    for res, v, want in [("cpu", 0, "0"), ("memory", 0, "0"), ("cpu", 1, "1m"), ("cpu", 1500, "1500m"),
                         ("cpu", 2000000, "2k"), ("memory", -2048, "-2Ki"), ("memory", 1023, "1023"),
                         ("memory", 1025, "1025"), ("hugepages-2Mi", 2 * 1024 * 1024, "2Mi"),
                         ("ephemeral-storage", 3 * 1024 ** 4, "3Ti"), ("pods", 110, "110"),
                         ("example.com/gpu", 8000, "8k"), ("memory", 2 ** 63 - 1, "9223372036854775807"),
                         ("pods", -(2 ** 63), "-9223372036854775808")]:
        assert native.resource_quantity_string(res, v, lib=lib) == want, (res, v)


@pytest.mark.parametrize("check", CHECKS, ids=lambda f: f.__name__)
def test_emulated(check, emu_lib):
    check(lambda d: TASFlavorSnapshot(d, lib=emu_lib))


@pytest.mark.gpu
@pytest.mark.parametrize("check", CHECKS, ids=lambda f: f.__name__)
def test_on_gpu(check):
    check(lambda d: TASFlavorSnapshot(d))
