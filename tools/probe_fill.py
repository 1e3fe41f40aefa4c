"""Diagnostic (profiling build, `make -C kueue_oss_amd/csrc prof`): where a
fill_pair_kernel block's time goes on the C3 batch.  Per block the kernel
stamps (100 MHz clock) its start, the records staged in LDS, CountIn done,
the leaf categories numbered, the verdicts settled, the class loop done;
this prints the medians / p90 of each phase and of the block's span, and the
spread of block start times (how the grid is dispatched)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kueue_oss_amd import TASFlavorSnapshot, native, synth  # noqa: E402

lib = native.load_library(os.path.join(os.path.dirname(native.library_path()), "libkueue_tas_prof.so"))
doc, wls = synth.CONFIGS[os.environ.get("CONFIG", "C3")](n_workloads=1024)
snap = TASFlavorSnapshot(doc, lib=lib)
snap.compile(wls)
for _ in range(3):
    snap.run_compiled()
buf = (ctypes.c_int32 * (1 << 18))()
k = lib.kueue_tas_last_fill_profile(snap.device_ctx(), buf, 1 << 18)
a = np.frombuffer(buf, dtype=np.int32, count=k).reshape(-1, 8).astype(np.int64)
a = a[a[:, 0] != 0]
t0 = a[:, 0].min()
names = ["staged", "countin", "categories", "verdicts", "class_loop"]
print("blocks", len(a), "kernel span us", (a[:, 5].max() - t0) / 100.0)
print("block start spread us: p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(
    np.percentile((a[:, 0] - t0) / 100.0, [10, 50, 90, 100])))
for i, n in enumerate(names):
    d = (a[:, i + 1] - a[:, i]) / 100.0
    print("%-12s median %.2f us  p90 %.2f  max %.2f" % (n, np.median(d), np.percentile(d, 90), d.max()))
span = (a[:, 5] - a[:, 0]) / 100.0
print("block span   median %.2f us  p90 %.2f  max %.2f" % (np.median(span), np.percentile(span, 90), span.max()))
print(snap.last_stats())
