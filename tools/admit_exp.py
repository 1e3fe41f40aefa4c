"""A/B of the admission pass on the C3 8,192-candidate round (the 8-GPU
rank-0 load, as bench.py extras.admission_8192): KTAS_ADMIT_PHASES values
given on the command line, each on a fresh snapshot; five timed rounds each
(the deltas negated after every round)."""
import json
import os
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from kueue_oss_amd import TASFlavorSnapshot, synth  # noqa: E402

doc, wls = synth.config_c3(n_workloads=8192)
ref = None
for ph in sys.argv[1:]:
    os.environ["KTAS_ADMIT_PHASES"] = ph
    snap = TASFlavorSnapshot(doc)
    snap.compile(wls)
    snap.run_compiled()
    quads = snap.last_assignments()
    rows = []
    for _ in range(6):
        t0 = time.perf_counter()
        admitted, deltas = snap.admit(quads)
        ms = (time.perf_counter() - t0) * 1e3
        rows.append((ms, snap.last_admit_times()))
        neg = deltas.copy()
        neg["delta"] = -neg["delta"]
        snap.apply_deltas(neg)
    key = (admitted.tolist(), np.sort(deltas, order=["leaf", "col"]).tobytes())
    assert ref is None or key == ref
    ref = key
    rows = rows[1:]
    print(json.dumps({"phases": ph, "round_ms": sorted(round(r[0], 3) for r in rows),
                      "device_ms": sorted(round(r[1][1], 3) for r in rows),
                      "prep_ms": sorted(round(r[1][0], 3) for r in rows), "stats": list(snap.last_admit_stats())}),
          flush=True)
    snap.close()
