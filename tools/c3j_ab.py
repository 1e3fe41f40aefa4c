"""A/B of two builds of the library on a bench batch (CONFIG, default C3J:
the multi-run fill): median fill and step over 12 runs each, alternating.
usage: [CONFIG=C3] python tools/c3j_ab.py <lib A> <lib B>"""
import sys
import time

sys.path.insert(0, ".")
from kueue_oss_amd import TASFlavorSnapshot, native, synth  # noqa: E402

import os  # noqa: E402

doc, wls = synth.CONFIGS[os.environ.get("CONFIG", "C3J")](n_workloads=1024)
libs = [native.load_library(p) for p in sys.argv[1:3]]
snaps = []
for lib in libs:
    s = TASFlavorSnapshot(doc, lib=lib)
    s.compile(wls)
    s.run_compiled()
    snaps.append(s)
ref = snaps[0].last_results()
assert snaps[1].last_results() == ref
res = [[], []]
for _ in range(12):
    for k, s in enumerate(snaps):
        t0 = time.perf_counter()
        s.run_compiled()
        st = s.last_stage_times()
        res[k].append(((time.perf_counter() - t0) * 1e3, st["fill"], st["select"], st["device_total"]))
for k, p in enumerate(sys.argv[1:3]):
    r = sorted(res[k])
    med = [sorted(x[i] for x in res[k])[len(r) // 2] for i in range(1, 4)]
    print(p, "step_ms", round(r[len(r) // 2][0], 3), "fill / select / device ms", [round(x, 3) for x in med])
