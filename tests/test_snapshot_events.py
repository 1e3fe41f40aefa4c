"""Device-resident snapshot maintenance: node events
(nodesCache.sync, tas_nodes_cache.go:38-72: in place for attribute updates,
a rebuild otherwise) and non-TAS pod events applied to a built snapshot in place (nonTasUsageCache.update/delete,
pkg/cache/scheduler/tas_non_tas_pod_cache.go:46-116, folded into the leaves'
freeCapacity as TASFlavorCache.snapshot does, tas_flavor.go:124-137) must give
the same evaluations as the reference's per-cycle rebuild — the oracle built
from scratch with the events appended to the snapshot's pod list, which it
replays through the same cache semantics (a terminated pod is the cache's
delete)."""
import copy
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth

GI = 1 << 30


def pod_events(rng, case, n):
    """Random pod events: new pods, replacements of known pods (node move,
    resize, new resource names), deletions, terminations, unknown nodes."""
    names = [nd["name"] for nd in case["nodes"]] or ["nowhere"]
    known = [(p["namespace"], p["name"]) for p in case.get("pods", [])]
    evs = []
    for k in range(n):
        r = rng.random()
        if known and r < 0.35:
            ns, name = rng.choice(known)
        else:
            ns, name = "ev", f"e{k}"
            known.append((ns, name))
        ev = {"namespace": ns, "name": name, "nodeName": rng.choice(names) if rng.random() < 0.95 else "ghost",
              "phase": rng.choice(["Running", "Running", "Running", "Pending", "Succeeded", "Failed"]), "requests": {}}
        for res in rng.sample(["cpu", "memory", "example.com/gpu", "example.com/new"], rng.randint(0, 3)):
            ev["requests"][res] = (rng.choice([0, 250, 1000, 4000]) if res == "cpu" else
                                   rng.choice([0, GI // 2, 2 * GI]) if res == "memory" else rng.choice([0, 1, 2]))
        if rng.random() < 0.15:
            ev["delete"] = True
        evs.append(ev)
    return evs


def node_events(rng, ref, n):
    """Random node events against the latest state of every node: allocatable
    changes (sometimes a new resource), taints copied from another node or
    new, label value changes, NotReady / cordon, new nodes, topology moves."""
    latest = {}
    for nd in ref["nodes"]:
        latest[nd["name"]] = nd
    names = list(latest)
    levels = ref["levels"]
    evs = []
    for k in range(n):
        if not names:
            break
        nd = copy.deepcopy(latest[rng.choice(names)])
        r = rng.random()
        if r < 0.3:
            for res in list(nd["allocatable"]):
                if rng.random() < 0.6:
                    nd["allocatable"][res] = max(0, nd["allocatable"][res] + rng.choice([-1, 1, 2]) *
                                                 (1000 if res == "cpu" else GI if res == "memory" else 1))
            if rng.random() < 0.1:
                nd["allocatable"]["example.com/new"] = rng.choice([0, 3])
        elif r < 0.5:
            other = latest[rng.choice(names)]
            nd["taints"] = copy.deepcopy(other.get("taints", [])) if rng.random() < 0.8 else \
                [{"key": f"t{k}", "value": "v", "effect": "NoSchedule"}]
        elif r < 0.7:
            key = rng.choice(["zone", "gpu-type"])
            if rng.random() < 0.2:
                nd["labels"].pop(key, None)
            else:
                nd["labels"][key] = rng.choice(["a", "b", "t1", "t2"]) if rng.random() < 0.9 else f"new{k}"
        elif r < 0.8:
            if rng.random() < 0.5:
                nd["conditions"] = [{"type": "Ready", "status": "False"}]
            else:
                nd["unschedulable"] = True
        elif r < 0.9:
            nd["name"] = f"new-node-{k}-{rng.randint(0, 1 << 20)}"
            # a third of new nodes join under the copied node's hostname (one
            # leaf, capacity only: leafDomain.node stays the first node)
            if "kubernetes.io/hostname" in nd["labels"] and rng.random() < 0.66:
                nd["labels"]["kubernetes.io/hostname"] = nd["name"]
        else:
            lvl = rng.choice(levels)
            nd["labels"][lvl] = nd["labels"].get(lvl, "") + "x"
        nd["conditions"] = nd.get("conditions") or [{"type": "Ready", "status": "True"}]
        latest[nd["name"]] = nd
        if nd["name"] not in names:
            names.append(nd["name"])
        evs.append(nd)
    return evs


def _oracle_pods(evs):
    return [dict(e, phase="Succeeded") if e.get("delete") else e for e in evs]


def _check(seed, n, lib=None, gen=None):
    rng = random.Random(seed)
    for i in range(n):
        case = (gen or synth.random_case)(rng)
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        ref = copy.deepcopy(case)
        ref.setdefault("pods", [])
        for step in range(3):
            evs = pod_events(rng, ref, rng.randint(1, 8))
            snap.update_pods(evs)
            ref["pods"] += _oracle_pods(evs)
            got = snap.find_topology_assignments_for_flavor(case["podSets"])
            want = oracle_lib.run_case(ref)["results"]
            assert got == want, (i, step, evs, got, want)
        snap.close()


def _check_nodes(seed, n, lib=None, gen=None):
    """Node events interleaved with pod events and admitted usage; the oracle
    rebuilds from the document with every event appended and replays the
    usage updates (a session) — the reference's per-cycle rebuild."""
    rng = random.Random(seed)
    rebuilt = inplace = 0
    for i in range(n):
        case = (gen or synth.random_case)(rng)
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        ref = copy.deepcopy(case)
        ref.setdefault("pods", [])
        adds = []
        for step in range(4):
            kind = rng.random()
            if kind < 0.6:
                evs = node_events(rng, ref, rng.randint(1, 4))
                if snap.update_nodes(evs):
                    rebuilt += 1
                else:
                    inplace += 1
                ref["nodes"] = ref["nodes"] + evs
            elif kind < 0.8:
                evs = pod_events(rng, ref, rng.randint(1, 4))
                snap.update_pods(evs)
                ref["pods"] += _oracle_pods(evs)
            else:
                res = oracle_lib.session(ref, adds + [{"op": "find", "podSets": case["podSets"]}])[-1]
                u = synth.usage_records(case["podSets"], res)
                if u:
                    snap.add_usage(u)
                    adds.append({"op": "add", "usage": u})
            got = snap.find_topology_assignments_for_flavor(case["podSets"])
            want = oracle_lib.session(ref, adds + [{"op": "find", "podSets": case["podSets"]}])[-1]
            assert got == want, (i, step, got, want)
        snap.close()
    assert rebuilt > 0 and inplace > 0, (rebuilt, inplace)


def test_emulated_node_events(emu_lib):  # noqa: F811
    _check_nodes(94, 60, lib=emu_lib)


@pytest.mark.gpu
def test_node_events_on_gpu():
    _check_nodes(95, 200)


def test_emulated_pod_events(emu_lib):  # noqa: F811
    _check(91, 60, lib=emu_lib)


@pytest.mark.gpu
def test_pod_events_on_gpu():
    _check(92, 200)


@pytest.mark.gpu
def test_pod_events_arith_on_gpu():
    _check(93, 100, gen=synth.arith_stress_case)


def _check_recolumn(lib=None):
    """Compiled workloads (kueue_tas_host_compile / run_compiled) stay correct
    when events change the snapshot's resource columns after compile: a pod
    with a resource no leaf had (sorting before "cpu", so existing column
    indices shift) and a usage update with another new resource."""
    snap_doc, wls = synth.config_c3(n_workloads=24, shape=(2, 2, 4, 8))
    snap = TASFlavorSnapshot(snap_doc, lib=lib) if lib else TASFlavorSnapshot(snap_doc)
    snap.compile(wls)
    ref = copy.deepcopy(snap_doc)
    snap.run_compiled()
    assert snap.last_results() == oracle_lib.eval_workloads(ref, wls)[0]
    node = ref["nodes"][3]["name"]
    ev = [{"namespace": "x", "name": "p-new", "nodeName": node, "phase": "Running",
           "requests": {"aaa.io/new": 1, "cpu": 1000}}]
    snap.update_pods(ev)
    ref["pods"] = ref["pods"] + ev
    snap.run_compiled()
    assert snap.last_results() == oracle_lib.eval_workloads(ref, wls)[0]
    host = ref["nodes"][5]["labels"]["kubernetes.io/hostname"]
    u = [{"values": [host], "singlePodRequests": {"aab.io/other": 2, "memory": 1 << 30}, "count": 1}]
    snap.add_usage(u)
    snap.run_compiled()
    want = [oracle_lib.session(ref, [{"op": "add", "usage": u}, {"op": "find", "podSets": w}])[-1] for w in wls]
    assert snap.last_results() == want
    snap.close()


def test_emulated_recolumn_after_compile(emu_lib):
    _check_recolumn(emu_lib)


@pytest.mark.gpu
def test_recolumn_after_compile_on_gpu():
    _check_recolumn()


def _check_leave_return(seed, n, lib=None):
    """Nodes leaving the snapshot (NotReady, cordoned) and coming back, while
    their parent domain keeps another node: applied in place (the leaf leaves
    and returns, kueue_tas_snapshot_set_leaf_live), never a rebuild; every
    evaluation equals the oracle rebuilt from the document with the events,
    with admitted usage added meanwhile (also on leaves that are out)."""
    rng = random.Random(seed)
    steps_total = 0
    for i in range(n):
        case = synth.random_case(rng)
        if case["levels"][-1] != "kubernetes.io/hostname" or len(case["levels"]) < 2 or not case["nodes"]:
            continue
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        ref = copy.deepcopy(case)
        adds = []
        out = {}  # node name -> its last Ready document
        for step in range(6):
            latest = {nd["name"]: nd for nd in ref["nodes"]}
            live = [nd for nd in latest.values()  # in the snapshot: nodesCache.find (util/tas/node.go:21-33)
                    if nd["conditions"] == [{"type": "Ready", "status": "True"}] and not nd["unschedulable"]
                    and nd["name"] not in out and all(k in nd["labels"] for k in case["levels"])
                    and all(nd["labels"].get(k, "") == v for k, v in case.get("nodeLabels", {}).items())]
            r = rng.random()
            ev = None
            if out and r < 0.4:
                name = rng.choice(sorted(out))
                ev = out.pop(name)
            elif r < 0.85 and live:
                nd = rng.choice(live)
                hosts = [x["labels"].get("kubernetes.io/hostname") for x in case["nodes"]]
                parent = [nd["labels"].get(k) for k in case["levels"][:-1]]
                # siblings: live nodes under the same parent that own their leaf (a hostname
                # shared by two nodes makes one leaf whose level values come from one of them)
                sib = [x for x in live if [x["labels"].get(k) for k in case["levels"][:-1]] == parent
                       and hosts.count(x["labels"].get("kubernetes.io/hostname")) == 1]
                host = nd["labels"].get("kubernetes.io/hostname")
                shared = hosts.count(host) > 1
                # (a hostname shared by two nodes: the leaf's level values come from one of
                # them, so its return may re-position the leaf — a rebuild, not checked here)
                if len(sib) >= 2 and not shared and all(k in nd["labels"] for k in case["levels"]):
                    out[nd["name"]] = copy.deepcopy(nd)
                    ev = copy.deepcopy(nd)
                    if rng.random() < 0.5:
                        ev["conditions"] = [{"type": "Ready", "status": "False"}]
                    else:
                        ev["unschedulable"] = True
            if ev is not None:
                assert snap.update_nodes([ev]) is False, (i, step, ev["name"])
                ref["nodes"] = ref["nodes"] + [ev]
            else:
                res = oracle_lib.session(ref, adds + [{"op": "find", "podSets": case["podSets"]}])[-1]
                u = synth.usage_records(case["podSets"], res)
                if u:
                    snap.add_usage(u)
                    adds.append({"op": "add", "usage": u})
            got = snap.find_topology_assignments_for_flavor(case["podSets"])
            want = oracle_lib.session(ref, adds + [{"op": "find", "podSets": case["podSets"]}])[-1]
            assert got == want, (i, step, got, want)
            steps_total += 1
        snap.close()
    assert steps_total > 50


def test_emulated_leave_return_in_place(emu_lib):  # noqa: F811
    _check_leave_return(31, 60, lib=emu_lib)


@pytest.mark.gpu
def test_leave_return_in_place_on_gpu():
    _check_leave_return(32, 200)


def _check_grow(seed, n, lib=None):
    """Nodes joining the snapshot — new hosts under existing racks, under a
    new rack or block, and members moving to another position — are spliced
    into the tree in place, never a rebuild; every evaluation equals the
    oracle rebuilt from the document with the events, with admitted usage
    (also on the joined leaves) added meanwhile."""
    rng = random.Random(seed)
    steps_total = 0
    spliced = reloaded = 0  # joins the device took by kueue_tas_snapshot_splice / by a reload
    for i in range(n):
        case = synth.random_case(rng)
        levels = case["levels"]
        if levels[-1] != "kubernetes.io/hostname" or not case["nodes"]:
            continue
        snap = TASFlavorSnapshot(case, lib=lib) if lib else TASFlavorSnapshot(case)
        ref = copy.deepcopy(case)
        adds = []
        for step in range(6):
            latest = {nd["name"]: nd for nd in ref["nodes"]}
            hosts = [nd["labels"].get("kubernetes.io/hostname") for nd in latest.values()]
            members = [nd for nd in latest.values()
                       if nd["conditions"] == [{"type": "Ready", "status": "True"}] and not nd["unschedulable"]
                       and all(k in nd["labels"] for k in levels)
                       and all(nd["labels"].get(k, "") == v for k, v in case.get("nodeLabels", {}).items())]
            r = rng.random()
            ev = None
            if members and r < 0.7:
                src = rng.choice(members)
                ev = copy.deepcopy(src)
                ev["labels"]["kubernetes.io/hostname"] = f"g{i}-{step}"
                ev["name"] = f"grow-{i}-{step}"
                k = rng.randrange(len(levels))  # levels above k keep src's values
                for lv in levels[k:-1]:
                    ev["labels"][lv] = f"{ev['labels'][lv]}-n{step}"
                if rng.random() < 0.3 and hosts.count(src["labels"]["kubernetes.io/hostname"]) == 1:
                    # a member moves: same node name at the new position (its old leaf
                    # leaves, which needs a live sibling; otherwise a rebuild — skip)
                    ev["name"] = src["name"]
                    parent = [src["labels"].get(x) for x in levels[:-1]]
                    # (a hostname shared by two nodes makes one leaf, placed by one of them)
                    sib = [x for x in members if [x["labels"].get(y) for y in levels[:-1]] == parent
                           and hosts.count(x["labels"].get("kubernetes.io/hostname")) == 1]
                    if len(sib) < 2:
                        ev["name"] = f"grow-{i}-{step}"
            if ev is not None:
                evs = [ev]
                if rng.random() < 0.4:  # one batch: more joins (merged together), then an
                    for x in range(rng.randint(1, 3)):  # update of a joined node (merged first)
                        e2 = copy.deepcopy(ev)
                        e2["name"] = f"grow-{i}-{step}-{x}"
                        e2["labels"]["kubernetes.io/hostname"] = f"g{i}-{step}-{x}"
                        if rng.random() < 0.5:
                            e2["labels"][levels[0]] = f"{e2['labels'][levels[0]]}-m{x}"
                        evs.append(e2)
                    if rng.random() < 0.5:
                        e3 = copy.deepcopy(evs[-1])
                        e3["allocatable"]["cpu"] = e3["allocatable"].get("cpu", 0) + 500
                        evs.append(e3)
                loads0, splices0 = snap.snapshot_counters()
                assert snap.update_nodes(evs) is False, (i, step, [e["name"] for e in evs])
                loads1, splices1 = snap.snapshot_counters()
                spliced += splices1 - splices0
                reloaded += loads1 - loads0
                ref["nodes"] = ref["nodes"] + evs
            else:
                res = oracle_lib.session(ref, adds + [{"op": "find", "podSets": case["podSets"]}])[-1]
                u = synth.usage_records(case["podSets"], res)
                if u:
                    snap.add_usage(u)
                    adds.append({"op": "add", "usage": u})
            got = snap.find_topology_assignments_for_flavor(case["podSets"])
            want = oracle_lib.session(ref, adds + [{"op": "find", "podSets": case["podSets"]}])[-1]
            assert got == want, (i, step, got, want)
            steps_total += 1
        snap.close()
    assert steps_total > 50
    # joins splice the device snapshot; a reload only for a new resource or label column
    assert spliced > 20 and reloaded < spliced / 4, (spliced, reloaded)


def _check_join_64(lib=None, shape=(2, 4, 16, 32)):
    """64 hosts joining existing racks of a C3-shaped snapshot (131,072 nodes at
    full size), admitted usage on the snapshot first: one splice, no reload,
    every result of a C3 batch equal to the oracle's on the grown document."""
    doc, wls = synth.config_c3(n_workloads=48, shape=shape)
    snap = TASFlavorSnapshot(doc, lib=lib) if lib else TASFlavorSnapshot(doc)
    snap.compile(wls)
    snap.run_compiled()
    admitted, deltas = snap.admit(snap.last_assignments())
    res = snap.last_results()
    ref = copy.deepcopy(doc)
    for i, ok in admitted.tolist():
        if ok:
            ref.setdefault("tasUsage", []).extend(synth.usage_records(wls[i], res[i]))
    N = len(doc["nodes"])
    joins = []
    for k in range(64):
        nd = copy.deepcopy(doc["nodes"][k * 983 % N])
        nd["name"] = f"{nd['name']}-join{k}"
        nd["labels"]["kubernetes.io/hostname"] = f"{nd['labels']['kubernetes.io/hostname']}-join{k}"
        joins.append(nd)
    loads0, splices0 = snap.snapshot_counters()
    assert snap.update_nodes(joins) is False
    assert snap.snapshot_counters() == (loads0, splices0 + 1)
    ref["nodes"] = ref["nodes"] + joins
    got = snap.find_topology_assignments_for_workloads(wls)
    assert snap.snapshot_counters() == (loads0, splices0 + 1)  # the evaluation did not reload either
    snap.close()
    want, _ = oracle_lib.eval_workloads(ref, wls, threads=8)
    assert got == want


def test_emulated_join_64_spliced(emu_lib):  # noqa: F811
    _check_join_64(emu_lib, shape=(1, 2, 8, 16))


@pytest.mark.gpu
def test_join_64_spliced_on_gpu():
    _check_join_64(shape=(4, 16, 64, 32))


def test_emulated_grow_in_place(emu_lib):  # noqa: F811
    _check_grow(41, 60, lib=emu_lib)


@pytest.mark.gpu
def test_grow_in_place_on_gpu():
    _check_grow(42, 200)
