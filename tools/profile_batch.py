"""Profiling driver: a bench batch (1024 workloads; CONFIG, default C3) evaluated 3 times."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, synth

snap_doc, wls = synth.CONFIGS[os.environ.get("CONFIG", "C3")](n_workloads=int(os.environ.get("N_WL", "1024")))
snap = TASFlavorSnapshot(snap_doc, category_fill=os.environ.get("NO_CAT") is None,
                         packed_entries=os.environ.get("PACKED") is not None)
snap.compile(wls)
for _ in range(3):
    snap.run_compiled()
print(snap.last_timings())
