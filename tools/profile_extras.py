"""Profiling driver for the widened rows on C3: batched preemption search
(16 candidates) and v1beta2 encoding of a batch, with host wall times."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, synth

snap_doc, wls = synth.config_c3(n_workloads=1024)
snap = TASFlavorSnapshot(snap_doc)
got = snap.find_topology_assignments_for_workloads(wls[:64])
cands = [c for c in (synth.usage_records(w, r) for w, r in zip(wls[:64], got)) if c][:16]
for c in cands:
    snap.add_usage(c)
pre = [dict(p, count=p.get("count", 1) * 4) for p in wls[0]]
print("records per candidate", [sum(1 for _ in c) for c in cands])
for _ in range(3):
    t0 = time.perf_counter()
    r = snap.preemption_search(pre, cands)
    print("preemption ms", (time.perf_counter() - t0) * 1e3, r["firstFit"], r["fillBackEvals"])
    print("profile", r["profileMs"])
snap.compile(wls)
snap.run_compiled()
for _ in range(3):
    t0 = time.perf_counter()
    snap.last_v1beta2(materialize=False)
    print("v1beta2 ms", (time.perf_counter() - t0) * 1e3)
