"""Writes tests/golden/tas_replacement.json: the reference's node-replacement
table test, hand-transcribed case by case (TASFlavorSnapshot
.FindTopologyAssignmentsForFlavor with WithWorkload of a workload whose
Status.UnhealthyNodes names a node of its admitted TopologyAssignment).

Source: /root/reference/pkg/cache/scheduler/tas_cache_test.go
  TestFindTopologyAssignmentsMultiLayerReplacement :6343-6697
    "replace unhealthy node in incomplete rack slice"                :6364-6411
    "replacement fails when no capacity in incomplete slice domain"  :6412-6461
    "3-layer: innermost broken domain confines replacement ..."      :6462-6563
    "2-layer: sliceSize=2 prevents scattered single-pod placement"   :6564-6626
  harness :6627-6697: TASMultiLayerTopology on, one PodSet "main" with
  SinglePodRequests cpu: 1000 and the case's count and topology request; the
  workload's admission holds the existing assignment (levels [hostname]) and
  UnhealthyNodes the case's node; topology "default"; NotReady nodes are not
  in the snapshot (nodesCache.sync).
"""
import json
import os

HOST = "kubernetes.io/hostname"
BLOCK, RACK, SWITCH = "cloud.com/topology-block", "cloud.com/topology-rack", "cloud.com/topology-switch"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "pkg/cache/scheduler/tas_cache_test.go"


def node(path, cpu_milli, ready=True):
    """testingnode.MakeNode("b1-r1-x1").Label(block).Label(rack)[.Label(switch)].Label(hostname)
    .StatusAllocatable(cpu, pods: 10).Ready()/NotReady()"""
    keys = [BLOCK, RACK, SWITCH] if len(path) == 4 else [BLOCK, RACK]
    labels = dict(zip(keys, path[:-1]))
    labels[HOST] = path[-1]
    return {"name": "-".join(path), "labels": labels, "allocatable": {"cpu": cpu_milli, "pods": 10},
            "taints": [], "unschedulable": False,
            "conditions": [{"type": "Ready", "status": "True" if ready else "False"}]}


def ta(pairs):  # MakeTopologyAssignment([hostname]).Domain(...)...
    return {"levels": [HOST], "domains": [{"values": [h], "count": c} for h, c in pairs]}


def tr(constraints):  # Required: block + PodsetSliceRequiredTopologyConstraints
    return {"required": BLOCK, "preferred": None, "unconstrained": None, "podSetSliceRequiredTopology": None,
            "podSetSliceSize": None,
            "podsetSliceRequiredTopologyConstraints": [{"topology": t, "size": s} for t, s in constraints]}


def case(name, lines, levels, nodes, existing, admission_count, unhealthy, topo, count, want_ta, want_reason):
    ps = {"name": "main", "count": count, "requests": {"cpu": 1000}, "topologyRequest": topo, "tolerations": [],
          "nodeSelector": None, "podSetGroupName": None,
          "wantAssignment": want_ta, "wantReason": want_reason}
    return {"name": name, "line": lines, "source": SRC, "featureGates": {"TASMultiLayerTopology": True},
            "levels": levels, "nodeLabels": {}, "topologyName": "default", "flavorTolerations": [],
            "tasUsage": [], "pods": [], "nodes": nodes, "podSets": [ps], "simulateEmpty": False,
            "workload": {"unhealthyNodes": [unhealthy], "admissionCount": admission_count,
                         "podSetAssignments": [{"name": "main", "topologyAssignment": existing}]}}


DEF = [BLOCK, RACK, HOST]
cases = [
    case("replace unhealthy node in incomplete rack slice", "6364-6411", DEF,
         [node(["b1", "r1", "x1"], 1000), node(["b1", "r1", "x2"], 1000), node(["b1", "r2", "x3"], 1000, False),
          node(["b1", "r2", "x4"], 1000), node(["b1", "r2", "x5"], 2000)],
         ta([("x1", 1), ("x2", 1), ("x3", 1), ("x4", 1)]), 4, "x3", tr([(RACK, 2)]), 4,
         ta([("x1", 1), ("x2", 1), ("x4", 2)]), ""),
    case("replacement fails when no capacity in incomplete slice domain", "6412-6461", DEF,
         [node(["b1", "r1", "x1"], 1000), node(["b1", "r1", "x2"], 1000), node(["b1", "r2", "x3"], 1000, False),
          node(["b1", "r2", "x4"], 500)],
         ta([("x1", 1), ("x2", 1), ("x3", 1), ("x4", 1)]), 4, "x3", tr([(RACK, 2)]), 4,
         None, 'topology "default" doesn\'t allow to fit any of 1 pod(s). Total nodes: 3; excluded: '
               'resource "cpu": 1, topologyDomain: 2'),
    case("3-layer: innermost broken domain confines replacement to correct switch", "6462-6563",
         [BLOCK, RACK, SWITCH, HOST],
         [node(["b1", "r1", "s1", "x1"], 4000), node(["b1", "r1", "s1", "x2"], 4000),
          node(["b1", "r1", "s2", "x3"], 4000, False), node(["b1", "r1", "s2", "x4"], 8000),
          node(["b1", "r2", "s3", "x5"], 4000), node(["b1", "r2", "s3", "x6"], 4000),
          node(["b1", "r2", "s4", "x7"], 4000), node(["b1", "r2", "s4", "x8"], 4000)],
         ta([(f"x{i}", 2) for i in range(1, 9)]), 16, "x3", tr([(RACK, 8), (SWITCH, 4), (HOST, 2)]), 16,
         ta([("x1", 2), ("x2", 2), ("x4", 4), ("x5", 2), ("x6", 2), ("x7", 2), ("x8", 2)]), ""),
    case("2-layer: sliceSize=2 prevents scattered single-pod placement across hosts", "6564-6626", DEF,
         [node(["b1", "r1", "x1"], 2000), node(["b1", "r1", "x2"], 2000), node(["b1", "r2", "x3"], 2000, False),
          node(["b1", "r2", "x4"], 1000), node(["b1", "r2", "x5"], 1000)],
         ta([("x1", 2), ("x2", 2), ("x3", 2), ("x4", 2)]), 8, "x3", tr([(RACK, 4), (HOST, 2)]), 8,
         None, 'topology "default" doesn\'t allow to fit any of 1 slice(s). Total nodes: 4; excluded: '
               'topologyDomain: 2'),
]

out = os.path.join(ROOT, "tests", "golden", "tas_replacement.json")
with open(out, "w") as f:
    json.dump({"source": SRC + ":6343-6697", "cases": cases}, f, indent=1)
print(out, len(cases))
