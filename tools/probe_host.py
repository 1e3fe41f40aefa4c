"""Diagnostic: host stages of the C3 bench step by run flags (precompiled,
+request compile, +TopologyAssignment values), medians over steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, synth

snap_doc, wls = synth.config_c3(n_workloads=1024)
snap = TASFlavorSnapshot(snap_doc)
snap.compile(wls)
C, V = TASFlavorSnapshot.RUN_COMPILE, TASFlavorSnapshot.RUN_VALUES
for name, fl in (("precompiled", 0), ("compile", C), ("values", V), ("full", C | V)):
    rows = []
    for i in range(40):
        t = time.perf_counter()
        snap.run_compiled(flags=fl)
        wall = (time.perf_counter() - t) * 1e3
        if i >= 10:
            rows.append([wall] + list(snap.last_profile()) + list(snap.last_device_host_times().values())
                        + list(snap.last_host_detail().values()))
    med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
    print(name, " ".join(f"{k}={v:.3f}" for k, v in zip(
        ["wall", "staging", "eval_call", "decode", "total", "d_compile", "d_classes", "d_enqueue", "d_wait", "d_pack",
         "d_copy", "d_validate", "d_records", "h_groups", "h_compile", "h_build_pass", "h_values"], med)))
res = snap.last_results()
print("failures", sum(1 for r in res for p in r if p["reason"]), "domains",
      sum(len(p["assignment"]["domains"]) for r in res for p in r if p.get("assignment")))
