"""Diagnostic: C3 stage times with the ExclusionStats counted inside the fill
(inline_stats) vs in fill_exclusion_kernel on a third stream (default)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, synth

snap_doc, wls = synth.config_c3(n_workloads=1024)
for inline in (False, True, False, True):
    snap = TASFlavorSnapshot(snap_doc, inline_stats=inline)
    snap.compile(wls)
    runs = []
    for _ in range(25):
        snap.run_compiled()
        runs.append(snap.last_stage_times())
    med = {k: round(sorted(r[k] for r in runs)[len(runs) // 2], 4) for k in runs[0]}
    print(json.dumps({"inline_stats": inline, **med}), flush=True)
    snap.close()
