"""Diagnostic: the C3J step (ragged racks, ~1,000 phase-1 classes) — median
wall ms and device stage ms over steps; `--check N` compares the first N
workloads with the oracle."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from kueue_oss_amd import TASFlavorSnapshot, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--check", type=int, default=0)
ap.add_argument("--config", default="C3J")
a = ap.parse_args()
doc, wls = synth.CONFIGS[a.config](n_workloads=1024)
snap = TASFlavorSnapshot(doc, category_fill=not os.environ.get("NO_CAT"))
snap.compile(wls)
FULL = TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES
for _ in range(3):
    snap.run_compiled(flags=FULL)
walls, stages = [], []
for _ in range(a.steps):
    t = time.perf_counter()
    snap.run_compiled(flags=FULL)
    walls.append((time.perf_counter() - t) * 1e3)
    stages.append(snap.last_stage_times())
med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
print(f"{a.config} env_ragged_pair={os.environ.get('KTAS_RAGGED_PAIR')} wall_ms={med(walls):.3f} "
      f"placements/s={1024 / med(walls) * 1e3:.0f} paths={snap.last_stats()['fill_paths']}")
print("stages_ms", {k: round(med([s[k] for s in stages]), 4) for k in stages[0]})
if a.check:
    import oracle_lib

    want, _ = oracle_lib.eval_workloads(doc, wls[: a.check], threads=16)
    got = snap.last_results()[: a.check]
    print("parity", got == want, [i for i in range(a.check) if got[i] != want[i]][:8])
snap.close()
