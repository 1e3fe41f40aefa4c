"""Admission round timing (rank 0's Fits + AddUsage in workload order,
kueue_tas_host_admit) for the gathered assignments of N workloads: the
Python-side total of TASFlavorSnapshot.admit beside the library's own parts
(host record prep, kueue_tas_admit, delta list), so the round's time is
attributed.  Each repetition's deltas are negated afterwards.

    python tools/probe_admit.py [CONFIG] [N ...]      (default: C3 1024 8192)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kueue_oss_amd import TASFlavorSnapshot, synth  # noqa: E402

FULL = TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "C3"
    sizes = [int(x) for x in sys.argv[2:]] or [1024, 8192]
    doc, wls = synth.CONFIGS[config](n_workloads=max(sizes))
    snap = TASFlavorSnapshot(doc, max_batch=1024)
    snap.compile(wls)
    out = {"config": config, "nodes": len(doc["nodes"]), "rounds": []}
    for n in sizes:
        snap.set_shard(list(range(n)))
        snap.run_compiled(flags=FULL)
        reps = []
        for r in range(6):
            t0 = time.perf_counter()
            quads = snap.last_assignments()
            t1 = time.perf_counter()
            admitted, deltas = snap.admit(quads)
            t2 = time.perf_counter()
            parts = snap.last_admit_times()
            stats = snap.last_admit_stats()
            neg = deltas.copy()
            neg["delta"] = -neg["delta"]
            snap.apply_deltas(neg)
            if r:  # the first repetition warms the buffers
                reps.append({"last_assignments_ms": (t1 - t0) * 1e3, "admit_ms": (t2 - t1) * 1e3,
                             "host_prep_ms": parts[0], "admit_device_ms": parts[1], "delta_list_ms": parts[2],
                             "window_rounds": stats[0], "in_order": stats[1]})
        med = {k: round(float(np.median([x[k] for x in reps])), 3) for k in reps[0]}
        med.update({"candidates": n, "quads": int(quads.size // 4), "admitted": int(admitted[:, 1].sum()),
                    "deltas": int(len(deltas))})
        med["unattributed_ms"] = round(med["admit_ms"] - med["host_prep_ms"] - med["admit_device_ms"]
                                       - med["delta_list_ms"], 3)
        out["rounds"].append(med)
        print(json.dumps(med), flush=True)
    snap.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
