"""Diagnostic: the host timeline of the C3 bench step (the full step,
RUN_COMPILE | RUN_VALUES): the host layer's stages and the device layer's
eval_chunk trace points (kueue_tas_last_host_trace), medians over steps."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kueue_oss_amd import TASFlavorSnapshot, synth

POINTS = ["validate", "layout", "records", "tables", "cls_merge", "cls_rep", "cls_order", "cls_members",
          "classes", "buffers", "fillpos", "upload", "fill_launch", "rollup_launch", "lfc_launch", "select_launch",
          "d2h_enq", "synced", "offsets"]
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
snap_doc, wls = synth.CONFIGS[cfg](n_workloads=1024)
snap = TASFlavorSnapshot(snap_doc)
snap.compile(wls)
lib = snap._lib
lib.kueue_tas_last_host_trace.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
ctx = snap.device_ctx()
FULL = TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES
snap.set_stage_timing(False)
rows = []
for i in range(61):
    t = time.perf_counter()
    snap.run_compiled(flags=FULL)
    wall = (time.perf_counter() - t) * 1e3
    tr = (ctypes.c_double * 20)()
    lib.kueue_tas_last_host_trace(ctx, tr, 20)
    if 10 <= i < 60:
        rows.append([wall] + list(snap.last_host_detail().values()) + list(tr)[1:20])
med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
names = ["wall"] + ["h_" + k for k in snap.last_host_detail()] + POINTS
print(cfg, " ".join(f"{k}={v:.3f}" for k, v in zip(names, med)))
