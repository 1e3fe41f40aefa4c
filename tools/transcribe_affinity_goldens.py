"""Writes tests/golden/tas_affinity.json: the reference's own fixtures for
required node affinity on the TAS path, hand-transcribed (the scheduler-level
table test is not parseable by tools/extract_goldens.py).

Source: /root/reference/pkg/scheduler/scheduler_tas_test.go (TestScheduleForTAS)
  :2618-2654 "does not admit workload when node does not match required affinity"
  :2655-2711 "admits workload when node matches required affinity"
with the shared objects of the same function:
  defaultSingleNode :66-77, defaultSingleLevelTopology :195
  (MakeDefaultOneLevelTopology = [kubernetes.io/hostname]),
  defaultTASFlavor :204-207 (nodeLabel tas-node=true, topology tas-single-level).

The scheduler test pins the outcome (inadmissible / the assignment); it
ignores the event message (eventIgnoreMessage), so the failure string of the
first case is recorded as derived ("wantReasonPinned": false): the oracle's
notFitMessage (tas_flavor_snapshot.go:1721-1741) with the Affinity exclusion
(:1605-1610).
"""
import json
import os

HOST = "kubernetes.io/hostname"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def node(name, labels, alloc):
    return {"name": name, "labels": labels, "allocatable": alloc, "taints": [], "unschedulable": False,
            "conditions": [{"type": "Ready", "status": "True"}]}


def affinity(key, values):
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": key, "operator": "In", "values": values}]}]}}}


GI = 1 << 30
ALLOC = {"cpu": 1000, "memory": GI, "pods": 10}  # StatusAllocatable cpu 1, memory 1Gi, pods 10


def podset(aff):
    # MakePodSet("one", 1).PreferredTopologyRequest(LabelHostname).Request(cpu, "1")
    return {"name": "one", "count": 1, "requests": {"cpu": 1000},
            "topologyRequest": {"preferred": HOST, "required": None, "unconstrained": None,
                                "podSetSliceRequiredTopology": None, "podSetSliceSize": None,
                                "podsetSliceRequiredTopologyConstraints": []},
            "tolerations": [], "nodeSelector": None, "podSetGroupName": None, "affinity": aff}


def case(name, line, nodes, ps, want_assignment, want_reason, pinned):
    ps = dict(ps, wantAssignment=want_assignment, wantReason=want_reason, wantReasonPinned=pinned)
    return {"name": name, "line": line, "scope": "in", "source": "pkg/scheduler/scheduler_tas_test.go",
            "featureGates": {}, "levels": [HOST], "nodeLabels": {"tas-node": "true"},
            "topologyName": "tas-single-level", "flavorTolerations": [], "tasUsage": [], "pods": [],
            "nodes": nodes, "podSets": [ps], "simulateEmpty": False}


def main():
    cases = [
        case("does not admit workload when node does not match required affinity", 2618,
             [node("x1", {"tas-node": "true", HOST: "x1"}, ALLOC)],
             podset(affinity("unused-key", ["value"])), None,
             'topology "tas-single-level" doesn\'t allow to fit any of 1 pod(s). Total nodes: 1; excluded: affinity: 1',
             False),
        case("admits workload when node matches required affinity", 2655,
             [node("x1", {"tas-node": "true", HOST: "x1", "expected-label": "expected-value"}, ALLOC)],
             podset(affinity("expected-label", ["expected-value"])),
             {"levels": [HOST], "domains": [{"values": ["x1"], "count": 1}]}, "", True),
    ]
    out = os.path.join(ROOT, "tests", "golden", "tas_affinity.json")
    with open(out, "w") as f:
        json.dump({"source": "pkg/scheduler/scheduler_tas_test.go:2618-2711 (hand transcription)",
                   "generator": "tools/transcribe_affinity_goldens.py", "cases": cases}, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
