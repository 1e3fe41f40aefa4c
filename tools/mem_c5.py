"""Device bytes of a 1M-node (C5) context after a 1,024-evaluation batch
(kueue_tas_device_bytes): every buffer, and the per-batch evaluation state."""
import json
import sys
import time

sys.path.insert(0, ".")
from kueue_oss_amd import TASFlavorSnapshot, synth  # noqa: E402

t0 = time.time()
doc, wls = synth.config_c5(n_workloads=1024)
snap = TASFlavorSnapshot(doc, max_batch=1024)
after_load = snap.device_bytes()
snap.compile(wls)
snap.run_compiled()
total, p2 = snap.device_bytes()
st = snap.last_stats()
print(json.dumps({"nodes": len(doc["nodes"]), "evals": len(wls), "after_load_bytes": after_load[0],
                  "total_bytes": total, "phase2_bytes": p2, "total_gb": round(total / 2**30, 2),
                  "phase2_gb": round(p2 / 2**30, 2), "stats": {k: st[k] for k in list(st)[:12]},
                  "seconds": round(time.time() - t0, 1)}))
snap.close()
