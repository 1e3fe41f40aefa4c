"""Diagnostic: per-eval select-kernel time on the C3 bench batch (which evals
form the kernel's critical path).  --prof loads the profiling build
(`make -C kueue_oss_amd/csrc prof` first: it is not part of build() and does
not ship with the tree unless built)."""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, native, synth

PROF = "--prof" in sys.argv
lib = native.load_library(os.path.join(os.path.dirname(native.library_path()), "libkueue_tas_prof.so")) if PROF else None

snap_doc, wls = synth.config_c3(n_workloads=int(os.environ.get("N_WL", "1024")))
if os.environ.get("BF_ONLY"):  # no unconstrained (fast-LFC) evals: no concurrent LFC branch
    wls = [w for w in wls if w[0]["topologyRequest"] is not None and not w[0]["topologyRequest"].get("unconstrained")]
snap = TASFlavorSnapshot(snap_doc, lib=lib, packed_entries=bool(os.environ.get("PACKED")),
                         host_values=bool(os.environ.get("HOST_VALUES")))
res = snap.find_topology_assignments_for_workloads(wls)
snap.compile(wls)
for _ in range(3):
    snap.run_compiled()
ticks = snap.last_eval_ticks(len(wls))
prof = snap.last_eval_profile(len(wls)) if PROF else None


def cls(w):
    tr = w[0]["topologyRequest"]
    if tr is None or tr.get("unconstrained"):
        return "unconstrained"
    return ("required:" + tr["required"].split("-")[-1]) if tr.get("required") else ("preferred:" + tr["preferred"].split("-")[-1])


rows = []
for i, w in enumerate(wls):
    r = res[i][0]
    nd = len(r["assignment"]["domains"]) if r.get("assignment") else 0
    rows.append({"i": i, "us": ticks[i][0] / 100.0, "find_us": ticks[i][1] / 100.0, "cls": cls(w), "count": w[0]["count"],
                 "req": w[0]["requests"], "sel": bool(w[0].get("nodeSelector")), "tol": bool(w[0].get("tolerations")),
                 "domains": nd, "fail": (r.get("reason") or "")[:60]})
    if PROF:
        rows[-1]["prof_us"] = {k: v / 100.0 for k, v in prof[i].items() if v}
rows.sort(key=lambda r: -r["us"])
for r in rows[:25]:
    print(json.dumps(r))
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["cls"], "fail" if r["fail"] else "ok")].append(r["us"])
for k, v in sorted(agg.items()):
    v.sort()
    print(k, "n=%d" % len(v), "median=%.1fus" % v[len(v) // 2], "max=%.1fus" % v[-1], "sum=%.0fus" % sum(v))
print("stages", snap.last_stage_times())
