"""Diagnostic: device/host time of the C3 batch split by request class."""
import sys, time, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, synth

snap_doc, wls = synth.config_c3(n_workloads=1024)
def cls(w):
    tr = w[0]['topologyRequest']
    if tr is None or tr.get('unconstrained'): return 'unconstrained'
    return 'required' if tr.get('required') else 'preferred'
snap = TASFlavorSnapshot(snap_doc)
groups = {'all': wls}
for c in ('unconstrained', 'required', 'preferred'):
    groups[c] = [w for w in wls if cls(w) == c]
for name, g in groups.items():
    snap.compile(g)
    for _ in range(2): snap.run_compiled()
    t = time.perf_counter(); snap.run_compiled(); wall = (time.perf_counter() - t) * 1e3
    ms, cnt = snap.last_timings()
    print(json.dumps({"class": name, "n": len(g), "wall_ms": round(wall, 2), "device_ms": [round(x, 2) for x in ms],
                      "host_ms": [round(x, 2) for x in snap.last_profile()],
                      "stages": {k: round(v, 3) for k, v in snap.last_stage_times().items()}}))
