"""Seeded synthetic TAS inputs.

* ``bench_config(name)`` — the BASELINE.json configs:
  C1 1,024 nodes / C2 16,384 / C3 131,072 / C4 65,536 JobSet / C5 1,048,576,
  modelled on the reference's perf generator (test/performance/scheduler/
  generator/topology_generator.go:64-157: zone/block/rack/hostname labels,
  unpadded names, 96 cpu / 256Gi / 110 pods per node).
* ``random_case(rng)`` — small randomized cases for differential tests
  against the CPU oracle: taints (Equal/Exists/Lt/Gt tolerations), node
  selectors, non-TAS pods (incl. over-subscription), TAS usage, leaders,
  slices, multi-layer constraints, implied/unconstrained/preferred/required
  requests, both TASProfileMixed settings.

Documents follow the fixture schema of tools/extract_goldens.py.
"""
from __future__ import annotations

import random

HOST = "kubernetes.io/hostname"
ZONE = "cloud.provider.com/topology-zone"
BLOCK = "cloud.provider.com/topology-block"
RACK = "cloud.provider.com/topology-rack"
GI = 1 << 30


def _node(name, labels, alloc, taints=(), ready=True):
    return {"name": name, "labels": labels, "allocatable": alloc, "taints": list(taints),
            "unschedulable": False, "conditions": [{"type": "Ready", "status": "True" if ready else "False"}]}


def _ps(name, count, requests, required=None, preferred=None, unconstrained=None, slice_topo=None,
        slice_size=None, constraints=None, group=None, tolerations=None, selector=None, implied=False):
    tr = None
    if any(v is not None for v in (required, preferred, unconstrained, slice_topo)) or constraints:
        tr = {"required": required, "preferred": preferred, "unconstrained": unconstrained,
              "podSetSliceRequiredTopology": slice_topo, "podSetSliceSize": slice_size,
              "podsetSliceRequiredTopologyConstraints": constraints or []}
    d = {"name": name, "topologyRequest": tr, "requests": requests, "count": count,
         "tolerations": tolerations or [], "nodeSelector": selector, "podSetGroupName": group}
    if tr is None and not implied:
        d["implied"] = False
    return d


# ----------------------------------------------------------------------------
# Benchmark configurations
# ----------------------------------------------------------------------------
def _tree_nodes(shape, labels_for, alloc_for, taints_for=None):
    nodes = []
    idx = 0
    import itertools
    for path in itertools.product(*[range(n) for n in shape]):
        nodes.append(_node(f"node-{'-'.join(map(str, path))}", labels_for(path), alloc_for(idx, path),
                           taints_for(idx, path) if taints_for else ()))
        idx += 1
    return nodes


def config_c1(seed=42):
    """C1: block/rack/hostname 4x16x16 = 1,024 nodes; one PodSet of 64 pods,
    cpu 8 + memory 32Gi, required rack; TAS usage u~U{0..6} pods per node."""
    rng = random.Random(seed)
    levels = [BLOCK, RACK, HOST]
    usage = []

    def labels(p):
        return {BLOCK: f"block-{p[0]}", RACK: f"rack-{p[0]}-{p[1]}", HOST: f"node-b{p[0]}-r{p[1]}-n{p[2]}"}

    nodes = _tree_nodes((4, 16, 16), labels, lambda i, p: {"cpu": 96000, "memory": 256 * GI, "pods": 110})
    for n in nodes:
        u = rng.randint(0, 6)
        if u:
            usage.append({"values": [n["labels"][HOST]], "singlePodRequests": {"cpu": 8000, "memory": 32 * GI},
                          "count": u})
    snap = {"levels": levels, "nodes": nodes, "pods": [], "tasUsage": usage, "nodeLabels": {}, "featureGates": {}}
    wl = [[_ps("main", 64, {"cpu": 8000, "memory": 32 * GI}, required=RACK)]]
    return snap, wl


def _mixed_workloads(rng, n, levels_req, lowest, highest):
    wls = []
    for i in range(n):
        r = rng.random()
        cpu = rng.choice([1, 2, 4, 8])
        req = {"cpu": cpu * 1000, "memory": 4 * GI * cpu}
        count = max(1, int(round(2 ** rng.uniform(0, 8))))
        if r < 0.4:
            lvl = levels_req[0] if rng.random() < 0.7 else levels_req[1]
            wls.append([_ps(f"ps{i}", count, req, required=lvl)])
        elif r < 0.8:
            lvl = rng.choice(levels_req)
            wls.append([_ps(f"ps{i}", count, req, preferred=lvl)])
        elif r < 0.9:
            wls.append([_ps(f"ps{i}", count, req, unconstrained=True)])
        else:
            # slice-only ("balanced" class of the perf generator): LFC at the highest level
            ss = rng.choice([1, 2, 4])
            count = max(ss, count - count % ss)
            wls.append([_ps(f"ps{i}", count, req, slice_topo=lowest, slice_size=ss)])
    return wls


def config_c2(seed=1234, n_workloads=1000, shape=(2, 8, 32, 32)):
    """C2: zone/block/rack/hostname 2x8x32x32 = 16,384 nodes; 1k workloads:
    40% required (70% rack / 30% block), 40% preferred, 20% unconstrained or
    slice-only; pod count log-uniform [1,256]; cpu in {1,2,4,8}, memory 4Gi/cpu."""
    rng = random.Random(seed)
    levels = [ZONE, BLOCK, RACK, HOST]

    def labels(p):
        return {ZONE: f"zone-{p[0]}", BLOCK: f"block-{p[0]}-{p[1]}", RACK: f"rack-{p[0]}-{p[1]}-{p[2]}",
                HOST: f"node-z{p[0]}-b{p[1]}-r{p[2]}-n{p[3]}"}

    nodes = _tree_nodes(shape, labels, lambda i, p: {"cpu": 96000, "memory": 256 * GI, "pods": 110})
    usage = []
    for n in nodes:
        u = rng.randint(0, 8)
        if u:
            usage.append({"values": [n["labels"][HOST]], "singlePodRequests": {"cpu": 8000, "memory": 16 * GI},
                          "count": u})
    snap = {"levels": levels, "nodes": nodes, "pods": [], "tasUsage": usage, "nodeLabels": {}, "featureGates": {}}
    return snap, _mixed_workloads(rng, n_workloads, [RACK, BLOCK], HOST, ZONE)


def config_c3(seed=7, n_workloads=1000, shape=(4, 16, 64, 32)):
    """C3: 4x16x64x32 = 131,072 nodes with cpu/memory/amd.com/gpu/ephemeral-storage,
    non-TAS usage on every node, TAS GPU usage g~U{0..8}, 10% gpu-maint NoSchedule
    + 2% NoExecute taints, gpu-type label; 50% required/preferred (BestFit),
    50% unconstrained (LeastFreeCapacity); 30% with nodeSelector, 20% tolerating."""
    rng = random.Random(seed)
    levels = [ZONE, BLOCK, RACK, HOST]

    def labels(p):
        return {ZONE: f"zone-{p[0]}", BLOCK: f"block-{p[0]}-{p[1]}", RACK: f"rack-{p[0]}-{p[1]}-{p[2]}",
                HOST: f"node-z{p[0]}-b{p[1]}-r{p[2]}-n{p[3]}",
                "cloud.provider.com/gpu-type": "abcd"[(p[2] * 7 + p[3]) % 4]}

    def taints(i, p):
        r = rng.random()
        if r < 0.10:
            return [{"key": "gpu-maint", "value": "true", "effect": "NoSchedule"}]
        if r < 0.12:
            return [{"key": "gpu-maint", "value": "true", "effect": "NoExecute"}]
        return []

    alloc = {"cpu": 192000, "memory": 1536 * GI, "amd.com/gpu": 8, "ephemeral-storage": 3500 * GI, "pods": 110}
    nodes = _tree_nodes(shape, labels, lambda i, p: dict(alloc), taints)
    pods = []
    usage = []
    for n in nodes:
        pods.append({"name": f"ds-{n['name']}", "namespace": "kube-system", "nodeName": n["name"],
                     "phase": "Running", "requests": {"cpu": 2000, "memory": 4 * GI}})
        g = rng.randint(0, 8)
        if g:
            usage.append({"values": [n["labels"][HOST]],
                          "singlePodRequests": {"cpu": 24000, "memory": 192 * GI, "amd.com/gpu": 1,
                                                "ephemeral-storage": 100 * GI}, "count": g})
    snap = {"levels": levels, "nodes": nodes, "pods": pods, "tasUsage": usage, "nodeLabels": {}, "featureGates": {}}
    wls = []
    for i in range(n_workloads):
        gpus = rng.randint(1, 8)
        req = {"cpu": 24000 * gpus, "memory": 192 * GI * gpus, "amd.com/gpu": gpus, "ephemeral-storage": 100 * GI * gpus}
        count = max(1, int(round(2 ** rng.uniform(0, 10))))
        sel = {"cloud.provider.com/gpu-type": rng.choice("abcd")} if rng.random() < 0.3 else None
        tol = [{"key": "gpu-maint", "operator": "Exists", "value": "", "effect": ""}] if rng.random() < 0.2 else []
        if rng.random() < 0.5:
            lvl = rng.choice([RACK, BLOCK])
            if rng.random() < 0.5:
                wls.append([_ps(f"ps{i}", count, req, required=lvl, selector=sel, tolerations=tol)])
            else:
                wls.append([_ps(f"ps{i}", count, req, preferred=lvl, selector=sel, tolerations=tol)])
        else:
            wls.append([_ps(f"ps{i}", count, req, unconstrained=True, selector=sel, tolerations=tol)])
    return snap, wls


def config_c3j(seed=8, n_workloads=1000, shape=(4, 16, 64), rack_sizes=(20, 44)):
    """C3 made adversarial: ragged racks (uniform in rack_sizes, mean 32, so
    ~131k nodes and no uniform fan-out) and per-workload jittered cpu/memory
    requests (every workload its own request signature and phase-1 class).
    Same node resources, usage, taints, labels and request mix as C3."""
    rng = random.Random(seed)
    levels = [ZONE, BLOCK, RACK, HOST]
    alloc = {"cpu": 192000, "memory": 1536 * GI, "amd.com/gpu": 8, "ephemeral-storage": 3500 * GI, "pods": 110}
    nodes, pods, usage = [], [], []
    for z in range(shape[0]):
        for b in range(shape[1]):
            for r in range(shape[2]):
                for n in range(rng.randint(*rack_sizes)):
                    name = f"node-{z}-{b}-{r}-{n}"
                    t = rng.random()
                    taints = ([{"key": "gpu-maint", "value": "true", "effect": "NoSchedule"}] if t < 0.10 else
                              [{"key": "gpu-maint", "value": "true", "effect": "NoExecute"}] if t < 0.12 else [])
                    labels = {ZONE: f"zone-{z}", BLOCK: f"block-{z}-{b}", RACK: f"rack-{z}-{b}-{r}",
                              HOST: f"node-z{z}-b{b}-r{r}-n{n}", "cloud.provider.com/gpu-type": "abcd"[(r * 7 + n) % 4]}
                    nodes.append(_node(name, labels, dict(alloc), taints))
                    pods.append({"name": f"ds-{name}", "namespace": "kube-system", "nodeName": name,
                                 "phase": "Running", "requests": {"cpu": 2000, "memory": 4 * GI}})
                    g = rng.randint(0, 8)
                    if g:
                        usage.append({"values": [labels[HOST]],
                                      "singlePodRequests": {"cpu": 24000, "memory": 192 * GI, "amd.com/gpu": 1,
                                                            "ephemeral-storage": 100 * GI}, "count": g})
    snap = {"levels": levels, "nodes": nodes, "pods": pods, "tasUsage": usage, "nodeLabels": {}, "featureGates": {}}
    wls = []
    for i in range(n_workloads):
        gpus = rng.randint(1, 8)
        req = {"cpu": 24000 * gpus - 250 * rng.randint(0, 40), "memory": 192 * GI * gpus - (1 << 26) * rng.randint(0, 63),
               "amd.com/gpu": gpus, "ephemeral-storage": 100 * GI * gpus}
        count = max(1, int(round(2 ** rng.uniform(0, 10))))
        sel = {"cloud.provider.com/gpu-type": rng.choice("abcd")} if rng.random() < 0.3 else None
        tol = [{"key": "gpu-maint", "operator": "Exists", "value": "", "effect": ""}] if rng.random() < 0.2 else []
        if rng.random() < 0.5:
            lvl = rng.choice([RACK, BLOCK])
            kw = {"required": lvl} if rng.random() < 0.5 else {"preferred": lvl}
            wls.append([_ps(f"ps{i}", count, req, selector=sel, tolerations=tol, **kw)])
        else:
            wls.append([_ps(f"ps{i}", count, req, unconstrained=True, selector=sel, tolerations=tol)])
    return snap, wls


def config_c4(seed=11, n_workloads=256, shape=(2, 16, 64, 32)):
    """C4: 2x16x64x32 = 65,536 nodes; JobSet-like workloads: a PodSet group
    {leader 1 pod cpu-only, workers 16-512 required block with 16-pod rack
    slices} plus an independent second PodSet (assumedUsage chaining)."""
    rng = random.Random(seed)
    levels = [ZONE, BLOCK, RACK, HOST]

    def labels(p):
        return {ZONE: f"zone-{p[0]}", BLOCK: f"block-{p[0]}-{p[1]}", RACK: f"rack-{p[0]}-{p[1]}-{p[2]}",
                HOST: f"node-z{p[0]}-b{p[1]}-r{p[2]}-n{p[3]}"}

    nodes = _tree_nodes(shape, labels, lambda i, p: {"cpu": 96000, "memory": 256 * GI, "pods": 110})
    usage = []
    for n in nodes:
        u = rng.randint(0, 10)
        if u:
            usage.append({"values": [n["labels"][HOST]], "singlePodRequests": {"cpu": 8000, "memory": 16 * GI},
                          "count": u})
    snap = {"levels": levels, "nodes": nodes, "pods": [], "tasUsage": usage, "nodeLabels": {}, "featureGates": {}}
    wls = []
    for i in range(n_workloads):
        workers = 16 * rng.randint(1, 32)
        wls.append([
            _ps("leader", 1, {"cpu": 1000}, required=BLOCK, group="g", slice_topo=RACK, slice_size=1),
            _ps("workers", workers, {"cpu": 4000, "memory": 8 * GI}, required=BLOCK, group="g",
                slice_topo=RACK, slice_size=16),
            _ps("aux", rng.randint(1, 64), {"cpu": 2000, "memory": 4 * GI}, preferred=RACK),
        ])
    return snap, wls


def config_c5(seed=5, n_workloads=100000, shape=(8, 32, 128, 32)):
    """C5: 8x32x128x32 = 1,048,576 nodes; 100k workloads with the C2 mix."""
    rng = random.Random(seed)
    levels = [ZONE, BLOCK, RACK, HOST]

    def labels(p):
        return {ZONE: f"zone-{p[0]}", BLOCK: f"block-{p[0]}-{p[1]}", RACK: f"rack-{p[0]}-{p[1]}-{p[2]}",
                HOST: f"node-z{p[0]}-b{p[1]}-r{p[2]}-n{p[3]}"}

    nodes = _tree_nodes(shape, labels, lambda i, p: {"cpu": 96000, "memory": 256 * GI, "pods": 110})
    snap = {"levels": levels, "nodes": nodes, "pods": [], "tasUsage": [], "nodeLabels": {}, "featureGates": {}}
    return snap, _mixed_workloads(rng, n_workloads, [RACK, BLOCK], HOST, ZONE)


CONFIGS = {"C1": config_c1, "C2": config_c2, "C3": config_c3, "C3J": config_c3j, "C4": config_c4, "C5": config_c5}


# ----------------------------------------------------------------------------
# Randomized differential cases
# ----------------------------------------------------------------------------
_TAINTS = [
    {"key": "gpu", "value": "present", "effect": "NoSchedule"},
    {"key": "maint", "value": "", "effect": "NoExecute"},
    {"key": "soft", "value": "x", "effect": "PreferNoSchedule"},
    {"key": "level", "value": "5", "effect": "NoSchedule"},
    {"key": "level", "value": "12", "effect": "NoExecute"},
]
_TOLS = [
    {"key": "gpu", "operator": "Equal", "value": "present", "effect": ""},
    {"key": "gpu", "operator": "Exists", "value": "", "effect": "NoSchedule"},
    {"key": "maint", "operator": "Exists", "value": "", "effect": ""},
    {"key": "", "operator": "Exists", "value": "", "effect": "NoExecute"},
    {"key": "level", "operator": "Gt", "value": "4", "effect": ""},
    {"key": "level", "operator": "Lt", "value": "10", "effect": ""},
    {"key": "level", "operator": "Lt", "value": "007", "effect": ""},
]


def random_case(rng: random.Random, max_nodes: int = 60, profile_mixed=None) -> dict:
    nlev = rng.choice([1, 2, 3, 3, 4])
    hostname = rng.random() < 0.75
    keys = ["dc", "block", "rack", "sub"]
    levels = keys[: nlev - 1 if hostname else nlev] + ([HOST] if hostname else [])
    if not levels:
        levels = [HOST]
    nn = rng.randint(0, max_nodes)
    fan = [rng.randint(1, 4) for _ in levels]
    res_names = ["cpu", "memory", "pods", "example.com/gpu"]
    nodes = []
    for i in range(nn):
        labels = {}
        for k in levels:
            if k == HOST:
                labels[k] = f"x{i}" if rng.random() < 0.97 else f"x{rng.randint(0, nn)}"
            else:
                labels[k] = f"{k[0]}{rng.randint(1, fan[levels.index(k)] * 3)}"
        if rng.random() < 0.05 and levels[0] != HOST:
            labels.pop(levels[0])  # missing level label: filtered by NodeMatchesFlavor
        if rng.random() < 0.5:
            labels["zone"] = rng.choice(["a", "b"])
        if rng.random() < 0.3:
            labels["gpu-type"] = rng.choice(["t1", "t2", "t3"])
        alloc = {}
        for r in res_names:
            if rng.random() < 0.85:
                if r == "cpu":
                    alloc[r] = rng.choice([0, 500, 1000, 2000, 4000, 8000, 16000])
                elif r == "memory":
                    alloc[r] = rng.choice([0, GI, 2 * GI, 8 * GI, 64 * GI])
                elif r == "pods":
                    alloc[r] = rng.choice([0, 1, 3, 10, 110])
                else:
                    alloc[r] = rng.choice([0, 1, 2, 4, 8])
        taints = [dict(t) for t in rng.sample(_TAINTS, rng.randint(0, 2))] if rng.random() < 0.3 else []
        n = _node(f"node{i}", labels, alloc, taints, ready=rng.random() < 0.95)
        n["unschedulable"] = rng.random() < 0.03
        nodes.append(n)
    pods = []
    for j in range(rng.randint(0, nn // 2 + 1)):
        if not nodes:
            break
        target = rng.choice(nodes)["name"] if rng.random() < 0.9 else ""
        pods.append({"name": f"p{j}", "namespace": "ns", "nodeName": target,
                     "phase": rng.choice(["Running", "Running", "Pending", "Succeeded", "Failed"]),
                     "requests": {r: rng.choice([0, 250, 1000, 3000]) if r == "cpu" else rng.choice([0, GI // 2, GI])
                                  for r in rng.sample(["cpu", "memory"], rng.randint(0, 2))}})
    usage = []
    for n in nodes:
        if rng.random() < 0.3:
            vals = [n["labels"].get(HOST, "")] if hostname else [n["labels"].get(k, "") for k in levels]
            usage.append({"values": vals, "singlePodRequests": {"cpu": rng.choice([0, 500, 1000]),
                                                                 "memory": rng.choice([0, GI // 4])},
                          "count": rng.randint(1, 4)})
    gates = {}
    if profile_mixed is not None:
        gates["TASProfileMixed"] = profile_mixed
    elif rng.random() < 0.3:
        gates["TASProfileMixed"] = False
    if rng.random() < 0.3:
        gates["TASMultiLayerTopology"] = True
    nodeLabels = {"zone": "a"} if rng.random() < 0.1 else {}
    flavor_tols = [dict(rng.choice(_TOLS))] if rng.random() < 0.1 else []
    podsets = []
    nps = rng.choice([1, 1, 1, 2, 2, 3])
    group_mode = nps >= 2 and rng.random() < 0.5
    for k in range(nps):
        req = {}
        for r in ["cpu", "memory", "example.com/gpu", "example.com/fpga"]:
            if rng.random() < (0.8 if r == "cpu" else 0.25):
                if r == "cpu":
                    req[r] = rng.choice([0, 100, 500, 1000, 2000])
                elif r == "memory":
                    req[r] = rng.choice([0, GI // 2, GI])
                else:
                    req[r] = rng.choice([0, 1, 2])
        if rng.random() < 0.05:
            req["pods"] = rng.choice([0, 1])
        kind = rng.random()
        lvl = rng.choice(levels)
        low_idx = rng.randrange(levels.index(lvl), len(levels))
        slice_lvl = levels[low_idx]
        ss = rng.choice([1, 1, 2, 3, 4])
        count = rng.choice([0, 1, 1, 2, 3, 4, 5, 8, 12, 20, 40])
        if ss > 1 and rng.random() < 0.8:
            count = ss * max(1, count // ss)
        kw = {}
        if kind < 0.3:
            kw["required"] = lvl
        elif kind < 0.55:
            kw["preferred"] = lvl
        elif kind < 0.7:
            kw["unconstrained"] = True
        elif kind < 0.8:
            pass  # implied (topologyRequest nil)
        else:
            kw["slice_topo"] = slice_lvl
            kw["slice_size"] = ss
        if kw and "slice_topo" not in kw and rng.random() < 0.35:
            kw["slice_topo"] = slice_lvl
            kw["slice_size"] = ss if rng.random() < 0.95 else None
        if kw and rng.random() < 0.15 and low_idx + 1 < len(levels):
            inner = levels[rng.randrange(low_idx + 1, len(levels))]
            inner_sz = rng.choice([d for d in range(1, ss + 1) if ss % d == 0])
            kw["constraints"] = [{"topology": slice_lvl, "size": ss}, {"topology": inner, "size": inner_sz}]
            kw.pop("slice_topo", None)
            kw.pop("slice_size", None)
        tol = [dict(t) for t in rng.sample(_TOLS, rng.randint(0, 2))] if rng.random() < 0.4 else []
        sel = None
        if rng.random() < 0.25:
            sel = {rng.choice(["zone", "gpu-type", "missing"]): rng.choice(["a", "b", "t1", "t2", "zz"])}
        elif rng.random() < 0.05:
            sel = {}
        group = "grp" if group_mode and k < 2 else None
        name = f"ps{k}"
        podsets.append(_ps(name, count, req, tolerations=tol, selector=sel, group=group,
                           implied=not kw, **kw))
    return {"name": "random", "levels": levels, "nodes": nodes, "pods": pods, "tasUsage": usage,
            "nodeLabels": nodeLabels, "flavorTolerations": flavor_tols, "featureGates": gates, "podSets": podsets}


def lfc_stress_case(rng: random.Random, n_nodes: int = 5000, n_workloads: int = 40, big: bool = True):
    """LeastFreeCapacity leaf-level stress: rack/hostname nodes whose free
    slot counts (cpu / 1 cpu request) span the exact histogram bins and, with
    ``big``, the overflow range (>= 127), over several 2,048-leaf chunks;
    unconstrained workloads sized to hit the single-leaf first fit, the
    greedy threshold inside the bins, inside the overflow range, and the
    not-fit failure.  Workloads share phase-1 classes (same request)."""
    levels = [RACK, HOST]
    nodes = []
    for i in range(n_nodes):
        r = rng.random()
        if big and r < 0.02:
            slots = rng.randint(127, 900)
        elif r < 0.25:
            slots = 0
        else:
            slots = rng.choice([1, 1, 1, 2, 2, 3, 5, 8, 40, 126])
        nodes.append(_node(f"n{i}", {RACK: f"r{i // 64}", HOST: f"n{i}"},
                           {"cpu": slots * 1000, "memory": 4096 * GI, "pods": 5000}))
    total = 0
    for n in nodes:
        total += n["allocatable"]["cpu"] // 1000
    wls = []
    for k in range(n_workloads):
        kind = rng.random()
        if kind < 0.2:
            count = rng.randint(0, 130)
        elif kind < 0.5:
            count = rng.randint(100, 3000)
        elif kind < 0.8:
            count = rng.randint(max(1, total - 3000), total)
        else:
            count = total + rng.randint(1, 50)
        ps = _ps("main", count, {"cpu": 1000}, unconstrained=True)
        wls.append([ps])
    snap = {"levels": levels, "nodes": nodes, "pods": [], "tasUsage": [], "nodeLabels": {}, "featureGates": {}}
    return snap, wls


_EXTREME_CAP = [0, 1, 2, 3, 7, 1000, (1 << 31) - 1, 1 << 31, (1 << 32) + 5, (1 << 33) - 1, 3 << 40,
                10 ** 18 + 7, 1 << 62, (1 << 63) - 1]
_EXTREME_REQ = [1, 2, 3, 5, 7, 10 ** 9 + 7, 1 << 20, (1 << 20) + 1, (1 << 31) + 3, 1 << 40, 3 << 40,
                (1 << 62) + 3, (1 << 63) - 1]


def arith_stress_case(rng: random.Random, max_nodes: int = 40) -> dict:
    """random_case with adversarial int64 quantities: capacities up to
    2^63-1, requests with non-power-of-two and huge divisors, usage above
    allocatable (negative free), so CountInWithLimitingResource
    (pkg/resources/requests.go:183-217: int64 Go division, int32 truncation,
    clamp at 0) and the per-pod usage products (requests.go:53-57) wrap the
    way Go does.  The kernels divide with host-computed multiply-high magic."""
    case = random_case(rng, max_nodes=max_nodes)
    big = "example.com/big"

    def pick(vals):
        return rng.choice(vals) if rng.random() < 0.8 else rng.randrange(1, 1 << 63)

    for n in case["nodes"]:
        if rng.random() < 0.9:
            n["allocatable"][big] = pick(_EXTREME_CAP)
        if "cpu" in n["allocatable"] and rng.random() < 0.5:
            n["allocatable"]["cpu"] = pick(_EXTREME_CAP)
    for p in case["pods"]:
        if rng.random() < 0.5:
            p["requests"][big] = rng.choice(_EXTREME_REQ + [0])
    for u in case["tasUsage"]:
        if rng.random() < 0.5:
            u["singlePodRequests"][big] = rng.choice(_EXTREME_REQ)
    for ps in case["podSets"]:
        if rng.random() < 0.7:
            ps["requests"][big] = pick(_EXTREME_REQ)
        if "cpu" in ps["requests"] and rng.random() < 0.3:
            ps["requests"]["cpu"] = pick(_EXTREME_REQ)
    case["name"] = "arith-stress"
    return case


def usage_records(podsets: list, results: list) -> list:
    """workload.TopologyDomainRequests records of the admitted assignments in
    `results` (ComputeTASNetUsage, flavorassigner.go:94-130: per domain, the
    PodSet's single-pod requests and the domain's pod count)."""
    by_name = {p["name"].lower(): p for p in podsets}
    recs = []
    for r in results:
        a = r.get("assignment")
        if not a:
            continue
        req = by_name.get(r["name"], {}).get("requests", {})
        for d in a["domains"]:
            recs.append({"values": d["values"], "singlePodRequests": dict(req), "count": d["count"]})
    return recs


def admission_ops(rng: random.Random, case: dict, first_results: list) -> list:
    """An admission-loop script for one snapshot (pkg/scheduler/scheduler.go:
    426-435: Fits re-check, AddUsage; preemption's SimulateUsageRemoval,
    clusterqueue_snapshot.go:85-92), interleaved with evaluations: find / fits /
    add / remove ops as run by tests on the oracle and the device."""
    ps = case["podSets"]
    u = usage_records(ps, first_results)
    half = u[: len(u) // 2]
    grown = [dict(r, count=r["count"] + rng.choice([1, 3, 1000])) for r in u]
    leaf_vals = [d["values"] for r in first_results if r.get("assignment") for d in r["assignment"]["domains"]]
    junk = [{"values": ["no-such-domain"], "singlePodRequests": {"cpu": 1}, "count": 1}]
    if leaf_vals:
        junk.append({"values": rng.choice(leaf_vals), "singlePodRequests": {"example.com/new": 2, "cpu": 0},
                     "count": 2})
        junk.append({"values": rng.choice(leaf_vals), "singlePodRequests": {}, "count": rng.choice([0, 1])})
    return [
        {"op": "find", "podSets": ps},
        {"op": "fits", "usage": u},
        {"op": "fits", "usage": grown},
        {"op": "add", "usage": u},
        {"op": "find", "podSets": ps},
        {"op": "fits", "usage": u},
        {"op": "remove", "usage": half},
        {"op": "find", "podSets": ps},
        {"op": "fits", "usage": junk[:1]},
        {"op": "fits", "usage": junk[1:]},
        {"op": "add", "usage": junk},
        {"op": "find", "podSets": ps},
        {"op": "remove", "usage": u},
        {"op": "add", "usage": half},
        {"op": "find", "podSets": ps, "simulateEmpty": True},
        {"op": "find", "podSets": ps},
        {"op": "fits", "usage": u},
    ]


def run_session(snap, ops: list) -> list:
    """Runs admission_ops on a TASFlavorSnapshot (the device path)."""
    out = []
    for op in ops:
        k = op["op"]
        if k == "find":
            out.append(snap.find_topology_assignments_for_flavor(op["podSets"], op.get("simulateEmpty", False)))
        elif k == "fits":
            out.append(snap.fits(op["usage"]))
        elif k == "add":
            snap.add_usage(op["usage"])
            out.append(None)
        elif k == "remove":
            snap.remove_usage(op["usage"])
            out.append(None)
        else:
            raise ValueError(k)
    return out


def random_internal_assignment(rng: random.Random):
    """An internal TopologyAssignment (pkg/util/tas/tas_assignment.go:30-38)
    whose level values share prefixes/suffixes, overlap ("ababa"/"aba"),
    repeat, or are empty — the cases fillSingleCompactSliceValues
    (tas_assignment.go:135-197) distinguishes.  None sometimes."""
    if rng.random() < 0.03:
        return None
    nl = rng.choice([1, 1, 2, 3, 4])
    levels = [f"l{k}" for k in range(nl)]
    n = rng.choice([0, 1, 2, 2, 3, 5, 8, 30, 200])
    alpha = rng.choice(["ab", "abc", "a.", "xyz-0123"])

    def word(m):
        return "".join(rng.choice(alpha) for _ in range(m))

    per_level = []
    for _ in range(nl):
        mode = rng.random()
        pre, suf = word(rng.randint(0, 4)), word(rng.randint(0, 4))
        base = word(rng.randint(0, 6))
        vals = []
        for _ in range(n):
            if mode < 0.2:
                vals.append(base)  # universal
            elif mode < 0.35:
                vals.append(rng.choice([base, base + word(1), base[: max(0, len(base) - 1)]]))
            else:
                vals.append(pre + word(rng.randint(0, 3)) + suf)
        per_level.append(vals)
    same = rng.random() < 0.5
    c0 = rng.randint(1, 9)
    domains = [{"values": [per_level[k][j] for k in range(nl)], "count": c0 if same else rng.randint(1, 9)}
               for j in range(n)]
    return {"levels": levels, "domains": domains}


_AFF_KEYS = ["zone", "gpu-type", "num", HOST, "rack", "missing"]


def _aff_expr(rng, node_names, valid=True):
    key = rng.choice(_AFF_KEYS)
    op = rng.choice(["In", "In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"])
    pool = {"zone": ["a", "b", "c"], "gpu-type": ["t1", "t2", "t9"], "num": ["1", "5", "12", "007", "x"],
            HOST: node_names[:6] + ["nope"], "rack": ["r1", "r2", "r3"], "missing": ["a"]}[key]
    if op in ("In", "NotIn"):
        values = rng.sample(pool, rng.randint(1, min(3, len(pool))))
    elif op in ("Exists", "DoesNotExist"):
        values = None if rng.random() < 0.5 else []
    else:
        values = [rng.choice(["0", "3", "6", "10", "-1", "+4", "9223372036854775807"])]
    if not valid:
        k = rng.random()
        if k < 0.3:
            op = rng.choice(["Foo", "", "in"])
        elif k < 0.5:
            key = rng.choice(["-bad", "a/b/c", "UPPER/x", "/x", "x" * 70, "ok.io/"])
        elif k < 0.7:
            values = [] if op in ("In", "NotIn") else ["a", "b"]
        elif k < 0.85:
            values = ["bad value!", "<x>"] if op in ("In", "NotIn") else ["1.5"]
        else:
            values = ["y" * 64]
    return {"key": key, "operator": op, "values": values}


def _aff_field(rng, node_names, valid=True):
    op = rng.choice(["In", "NotIn"])
    key = "metadata.name" if rng.random() < 0.85 else "spec.other"
    v = rng.choice(node_names + ["", "ghost"]) if node_names else rng.choice(["", "ghost"])
    values = [v]
    if not valid:
        if rng.random() < 0.5:
            op = rng.choice(["Exists", "Gt"])
        else:
            values = [v, "other"] if rng.random() < 0.5 else []
    return {"key": key, "operator": op, "values": values}


def random_affinity(rng: random.Random, node_names: list, invalid_p: float = 0.1):
    """PodSpec affinity with required node affinity (nodeSelectorTerms ORed,
    matchExpressions / matchFields ANDed; nodeaffinity.go:84-201): label
    operators In/NotIn/Exists/DoesNotExist/Gt/Lt on present, absent and
    numeric labels, metadata.name fields, empty terms, an empty term list,
    and (with probability invalid_p) one malformed requirement whose
    validation error becomes the failure reason (tas_flavor_snapshot.go:889-897)."""
    terms = []
    for _ in range(rng.choice([0, 1, 1, 1, 2, 2, 3])):
        r = rng.random()
        t = {}
        if r < 0.08:
            pass  # empty term: skipped
        else:
            if r < 0.85:
                t["matchExpressions"] = [_aff_expr(rng, node_names) for _ in range(rng.randint(1, 3))]
            if r >= 0.6:
                t["matchFields"] = [_aff_field(rng, node_names) for _ in range(rng.randint(1, 2))]
        terms.append(t)
    if terms and rng.random() < invalid_p:
        t = rng.choice(terms)
        if rng.random() < 0.7:
            t.setdefault("matchExpressions", []).append(_aff_expr(rng, node_names, valid=False))
        else:
            t.setdefault("matchFields", []).append(_aff_field(rng, node_names, valid=False))
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": terms}}}


def affinity_case(rng: random.Random, max_nodes: int = 60, invalid_p: float = 0.1) -> dict:
    """random_case whose nodes carry a numeric label ("num") and whose PodSets
    set required node affinity (and sometimes an invalid nodeSelector)."""
    case = random_case(rng, max_nodes=max_nodes)
    for n in case["nodes"]:
        if rng.random() < 0.6:
            n["labels"]["num"] = rng.choice(["0", "2", "5", "11", "-3", "+7", "08", "abc"])
        if rng.random() < 0.03:
            n["name"] = ""
    names = [n["name"] for n in case["nodes"] if n["name"]]
    for ps in case["podSets"]:
        r = rng.random()
        if r < 0.8:
            ps["affinity"] = random_affinity(rng, names, invalid_p)
        elif r < 0.85:
            ps["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": None}}
        if rng.random() < invalid_p / 2:
            ps["nodeSelector"] = {rng.choice(["-bad", "ok", "a/b/c"]): rng.choice(["v!", "fine", ""])}
    case["name"] = "affinity"
    return case


_WIDE_EFFECTS = ["NoSchedule", "NoExecute", "PreferNoSchedule"]


def wide_case(rng: random.Random, variant: str, n_nodes: int = 400, n_workloads: int = 48):
    """Batches that reach the fill-kernel variants the bench configs never
    touch (tas_device.hip eval_chunk dispatch):

    * ``"cols"``: the batch's requests span 9..27 resource columns (up to 21
      terms in one request: ``fill_leaves_kernel<16>`` / ``<32>``), with many
      taint strings, so ``3 + taints + R > 64`` ExclusionStats slots take the
      global-atomic path;
    * ``"profiles"``: at most 5 request columns (the staged fill) and more
      than 32 distinct taint profiles: taint rows read from global memory and
      ``fill_exclusion_kernel<false>``;
    * ``"slots"``: at most 5 request columns and more than 61 taint strings:
      the staged fill counting ExclusionStats with global atomics;
    * ``"manyres"``: nodes with 47 resource names (more than
      KUEUE_TAS_MAX_COLS device columns), requests naming a few of them.

    Every variant has twelve label columns (selector columns beyond the four
    held in registers), nodeSelectors of up to 12 pairs (beyond the 8 inline
    pairs of kueue_tas_eval_req), required node affinity, tolerations
    (Equal / Exists / Gt / Lt) over the taint pool, leader / worker groups,
    slices and ragged racks.  Returns (snapshot document, workloads)."""
    levels = ["block", "rack", HOST]
    n_ext = {"cols": 24, "profiles": 2, "slots": 2, "manyres": 44}[variant]
    ext = [f"example.com/r{k:02d}" for k in range(n_ext)]
    n_tkeys = {"cols": 30, "profiles": 12, "slots": 40, "manyres": 3}[variant]
    pool = []
    for k in range(n_tkeys):
        for v in (["", "a"] if variant != "slots" else ["", "a", "7"]):
            pool.append({"key": f"t{k}", "value": v, "effect": _WIDE_EFFECTS[k % 3]})
    if variant == "slots":
        pool += [{"key": "lvl", "value": str(j), "effect": "NoSchedule"} for j in (1, 4, 9, 16, 25)]
    label_vals = {f"l{k}": [f"v{j}" for j in range(2 + k % 3)] for k in range(12)}
    nodes = []
    i = 0
    while i < n_nodes:
        b = rng.randrange(3)
        r = rng.randrange(6)
        for _ in range(rng.randint(1, 40)):
            if i >= n_nodes:
                break
            labels = {"block": f"b{b}", "rack": f"b{b}-r{r}", HOST: f"n{i}"}
            for key, vals in label_vals.items():
                if rng.random() < 0.85:
                    labels[key] = rng.choice(vals)
            alloc = {"cpu": rng.choice([0, 4000, 16000, 64000]), "memory": rng.choice([4 * GI, 64 * GI]), "pods": 110}
            for e in ext:
                if rng.random() < (0.97 if variant in ("cols", "manyres") else 0.8):
                    alloc[e] = rng.choice([0, 2, 4, 8, 16] if variant == "cols" else [0, 1, 2, 4, 8, 16])
            nt = rng.choice([0, 0, 0, 1, 2]) if variant == "cols" else rng.choice([0, 0, 1, 1, 2, 3])
            taints = [dict(t) for t in rng.sample(pool, nt)]
            nodes.append(_node(f"node{i}", labels, alloc, taints, ready=rng.random() < 0.97))
            i += 1
    tols_pool = [{"key": f"t{k}", "operator": rng.choice(["Exists", "Equal"]), "value": "a" if k % 2 else "",
                  "effect": rng.choice(["", _WIDE_EFFECTS[k % 3]])} for k in range(n_tkeys)]
    tols_pool += [{"key": "lvl", "operator": "Gt", "value": "5", "effect": ""},
                  {"key": "lvl", "operator": "Lt", "value": "10", "effect": ""}]
    names = [n["name"] for n in nodes]
    kmax = rng.choice([14, 21])  # longest request (+ pods): fill_leaves_kernel<16> or <32>
    wls = []
    for w in range(n_workloads):
        def podset(name, count, group=None):
            req = {"cpu": rng.choice([0, 500, 2000])} if rng.random() < 0.8 else {}
            if rng.random() < 0.5:
                req["memory"] = rng.choice([GI, 4 * GI])
            if variant == "cols":
                k = rng.choice([2, 6, 10, 13]) if w % 3 or kmax < 16 else rng.choice([18, 20, kmax])
                for e in rng.sample(ext, min(k, len(ext))):
                    req[e] = rng.choice([0, 1, 1, 1, 2])
            elif variant == "manyres":  # a few of the 44 node resources per request
                for e in rng.sample(ext[:12], rng.randint(0, 4)):
                    req[e] = rng.choice([0, 1, 2])
            else:
                for e in ext:
                    if rng.random() < 0.4:
                        req[e] = rng.choice([0, 1, 2])
            kind = rng.random()
            kw = {}
            if kind < 0.35:
                kw["required"] = rng.choice(levels[:2])
            elif kind < 0.6:
                kw["preferred"] = rng.choice(levels[:2])
            elif kind < 0.85:
                kw["unconstrained"] = True
            if kw and rng.random() < 0.25:
                kw["slice_topo"] = rng.choice(levels[1:])
                kw["slice_size"] = rng.choice([1, 2, 4])
                count = kw["slice_size"] * max(1, count // kw["slice_size"])
            sel = None
            if rng.random() < 0.6:  # mostly copied from a node's labels, so some nodes match
                keys = rng.sample(sorted(label_vals), rng.choice([1, 3, 8, 9, 10, 12]))
                like = rng.choice(nodes)["labels"]
                sel = {k: like[k] if k in like and rng.random() < 0.9 else rng.choice(label_vals[k]) for k in keys}
                if rng.random() < 0.05:
                    sel["absent-key"] = "x"
            tols = [dict(t) for t in rng.sample(tols_pool, rng.randint(0, min(6, len(tols_pool))))] if rng.random() < 0.7 else []
            ps = _ps(name, count, req, tolerations=tols, selector=sel, group=group, implied=not kw, **kw)
            if rng.random() < 0.2:
                ps["affinity"] = random_affinity(rng, names, invalid_p=0.0)
            return ps

        if rng.random() < 0.2:
            wls.append([podset("leader", 1, "g"), podset("workers", rng.choice([2, 4, 8]), "g")])
        else:
            wls.append([podset("main", rng.choice([1, 2, 3, 5, 8, 16, 40]))])
    snap = {"name": f"wide-{variant}", "levels": levels, "nodes": nodes, "pods": [], "tasUsage": [],
            "nodeLabels": {}, "featureGates": {}}
    return snap, wls


def balanced_case(rng: random.Random, max_nodes: int = 60) -> dict:
    """random_case under the TASBalancedPlacement gate (tas_flavor_snapshot.go:
    906-917) with mostly preferred requests (the gated branch), slices,
    leader groups and multi-layer constraints."""
    case = random_case(rng, max_nodes=max_nodes)
    case["featureGates"]["TASBalancedPlacement"] = True
    levels = case["levels"]
    for ps in case["podSets"]:
        tr = ps.get("topologyRequest")
        if tr is not None and tr.get("required") and rng.random() < 0.7:
            tr["preferred"], tr["required"] = tr["required"], None
        elif tr is None and rng.random() < 0.6:
            ps["topologyRequest"] = {"required": None, "preferred": rng.choice(levels), "unconstrained": None,
                                     "podSetSliceRequiredTopology": None, "podSetSliceSize": None,
                                     "podsetSliceRequiredTopologyConstraints": []}
            ps.pop("implied", None)
    case["name"] = "balanced"
    return case


def replacement_case(rng: random.Random, oracle_run) -> dict:
    """A node-replacement case (FindTopologyAssignmentsForFlavor with a
    workload whose Status.UnhealthyNodes names a node of its admitted
    assignment, tas_flavor_snapshot.go:546-562): the PodSets' existing
    assignments come from evaluating them first (`oracle_run(case)` ->
    results); the unhealthy node then usually leaves the snapshot
    (NotReady), sometimes a second assigned node too (a stale assignment),
    and the admitted usage is sometimes in the snapshot."""
    four = rng.random() < 0.35
    levels = ["block", "rack"] + (["switch"] if four else []) + [HOST]
    nodes = []
    for b in range(rng.randint(1, 3)):
        for r in range(rng.randint(1, 3)):
            for sw in range(rng.randint(1, 2) if four else 1):
                for k in range(rng.randint(1, 4)):
                    name = f"b{b}r{r}s{sw}x{k}"
                    labels = {"block": f"b{b}", "rack": f"b{b}-r{r}", HOST: name}
                    if four:
                        labels["switch"] = f"b{b}-r{r}-s{sw}"
                    nodes.append(_node(name, labels, {"cpu": rng.choice([1000, 2000, 4000, 8000]),
                                                      "pods": rng.choice([10, 110])}))
    gates = {"TASMultiLayerTopology": True} if rng.random() < 0.7 else {}
    podsets = []
    for k in range(rng.choice([1, 1, 2])):
        kind = rng.random()
        kw = {}
        lvl = rng.choice(levels[:-1])
        if kind < 0.45:
            kw["required"] = lvl
        elif kind < 0.7:
            kw["preferred"] = lvl
        elif kind < 0.8:
            kw["unconstrained"] = True
        count = rng.choice([1, 2, 3, 4, 6, 8])
        if kw and rng.random() < 0.6:
            inner = levels[levels.index(lvl) + 1:]
            a = rng.choice([1, 2, 4])
            cons = [{"topology": rng.choice(inner), "size": a}]
            if len(inner) > 1 and rng.random() < 0.5:
                li = levels.index(cons[0]["topology"])
                if li + 1 < len(levels):
                    cons.append({"topology": rng.choice(levels[li + 1:]), "size": rng.choice([d for d in (1, 2) if a % d == 0])})
            count = a * rng.randint(1, 4)
            if rng.random() < 0.5:
                kw["constraints"] = cons
            else:
                kw["slice_topo"], kw["slice_size"] = cons[0]["topology"], a
        podsets.append(_ps(f"ps{k}", count, {"cpu": rng.choice([500, 1000, 2000])}, implied=not kw, **kw))
    case = {"name": "replacement", "levels": levels, "nodes": nodes, "pods": [], "tasUsage": [], "nodeLabels": {},
            "flavorTolerations": [], "featureGates": gates, "podSets": podsets, "simulateEmpty": False}
    first = oracle_run(case)
    psa, assigned = [], []
    for r in first:
        if r["assignment"]:
            psa.append({"name": r["name"], "topologyAssignment": r["assignment"]})
            assigned += [d["values"][-1] for d in r["assignment"]["domains"]]
    if not assigned:
        return None
    unhealthy = rng.choice(assigned) if rng.random() < 0.9 else rng.choice([n["name"] for n in nodes])
    down = {unhealthy} if rng.random() < 0.85 else set()
    if rng.random() < 0.1:
        down.add(rng.choice(assigned))  # a second node gone: the assignment is stale
    for n in nodes:
        if n["labels"][HOST] in down:
            n["conditions"] = [{"type": "Ready", "status": "False"}]
    if rng.random() < 0.5:  # the admitted usage of the healthy domains is in the snapshot
        case["tasUsage"] = [u for u in usage_records(podsets, first) if u["values"][-1] not in down]
    case["workload"] = {"unhealthyNodes": [unhealthy], "podSetAssignments": psa}
    return case


def elastic_case(rng: random.Random, oracle_run) -> dict:
    """An elastic workload-slice case (ElasticJobsViaWorkloadSlicesWithTAS,
    tas_elastic_workloads.go:35-127): a random case whose PodSets were first
    placed (`oracle_run(case)` with the gate off) and now ask for more, fewer
    or the same pods with that placement as PreviousAssignment; sometimes a
    node of it has left the snapshot (stale: fresh placement)."""
    while True:
        case = random_case(rng, max_nodes=40)
        case["featureGates"] = dict(case["featureGates"])
        case["featureGates"].pop("ElasticJobsViaWorkloadSlicesWithTAS", None)
        first = oracle_run(case)
        placed = {r["name"]: r["assignment"] for r in first if r["assignment"] and r["assignment"]["domains"]}
        if placed:
            break
    for ps in case["podSets"]:
        a = placed.get(ps["name"])
        if a is None or rng.random() < 0.15:
            continue
        ps["previousAssignment"] = a
        prev = sum(d["count"] for d in a["domains"])
        ps["count"] = max(0, prev + rng.choice([-3, -1, 0, 0, 1, 2, 4, 8]))
    if rng.random() < 0.1:  # a previously used node leaves: stale, fresh placement
        used = {d["values"][-1] for a in placed.values() for d in a["domains"]}
        for n in case["nodes"]:
            if n["labels"].get(HOST) in used:
                n["conditions"] = [{"type": "Ready", "status": "False"}]
                break
    case["featureGates"]["ElasticJobsViaWorkloadSlicesWithTAS"] = True
    return case
