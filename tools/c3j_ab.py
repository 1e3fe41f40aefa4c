"""A/B of two builds of the library on the C3J batch (the multi-run fill):
median fill and step over 12 runs each, alternating.  usage:
python tools/c3j_ab.py <lib A> <lib B>"""
import sys
import time

sys.path.insert(0, ".")
from kueue_oss_amd import TASFlavorSnapshot, native, synth  # noqa: E402

doc, wls = synth.config_c3j(n_workloads=1024)
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
        res[k].append(((time.perf_counter() - t0) * 1e3, s.last_stage_times()["fill"]))
for k, p in enumerate(sys.argv[1:3]):
    r = sorted(res[k])
    f = sorted(x[1] for x in res[k])
    print(p, "step_ms", round(r[len(r) // 2][0], 3), "fill_ms", round(f[len(f) // 2], 3))
