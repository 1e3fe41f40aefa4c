"""Builds experiment variants of the library (patched copies under _exp/,
never the product) and times the fill stage of the C3 batch with each:

    python tools/exp_fill.py build      # here (hipcc cross-compiles)
    python tools/exp_fill.py run        # on the GPU box

Each variant removes one piece of fill_leaves_staged_kernel's per-eval loop
(results are then wrong: timing only) to show where the loop's time goes."""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXP = os.path.join(ROOT, "_exp")
K = "tas_kernels.hip"
VARIANTS = {
    "base": [],
    "no_loop": [("  for (int e = 0; e < ne; e++) {\n    const int4* pq",
                 "  for (int e = 0; e < (state0 == -7 ? ne : 0); e++) {\n    const int4* pq")],
    "no_excl": [("    if (valid && kind == EX_NONE) {\n      if (s.lowest_is_hostname) {\n        if (s.taint_profile) {\n          int t;",
                 "    if (valid && kind == EX_NONE) {\n      if (false) {\n        if (s.taint_profile) {\n          int t;")],
    "no_rack": [("  const int rack_f = b.rack_fanout;", "  const int rack_f = 0;")],
    "no_leaf_store": [("    if (valid) {\n      base[gleaf] = state;", "    if (valid && state == -7) {\n      base[gleaf] = state;")],
    "no_loop_no_count": [("  for (int e = 0; e < ne; e++) {\n    const int4* pq",
                          "  for (int e = 0; e < (state0 == -7 ? ne : 0); e++) {\n    const int4* pq"),
                         ("  if constexpr (!MR) count_run(0);", "  if constexpr (!MR) { if (ne < 0) count_run(0); }")],
    "no_count": [("  if constexpr (!MR) count_run(0);", "  if constexpr (!MR) { if (ne < 0) count_run(0); }")],
    "evals_per_block_8": [("constexpr int kEvalsPerBlock = 16;", "constexpr int kEvalsPerBlock = 8;")],
    "evals_per_block_32": [("constexpr int kEvalsPerBlock = 16;", "constexpr int kEvalsPerBlock = 32;")],
    "no_store_no_rack": [("    if (valid) {\n      base[gleaf] = state;", "    if (valid && state == -7) {\n      base[gleaf] = state;"),
                         ("  const int rack_f = b.rack_fanout;", "  const int rack_f = 0;")],
}


def build():
    src = os.path.join(ROOT, "kueue_oss_amd", "csrc")
    for name, patches in VARIANTS.items():
        d = os.path.join(EXP, name)
        shutil.rmtree(d, ignore_errors=True)
        shutil.copytree(src, os.path.join(d, "csrc"))
        os.makedirs(os.path.join(d, "include"), exist_ok=True)
        for h in ("kueue_tas.h", "kueue_tas_debug.h"):
            shutil.copy(os.path.join(ROOT, "include", h), os.path.join(d, "include", h))
        # the sources include "../../include/..." -> point at the copy
        p = os.path.join(d, "csrc", K)
        s = open(p).read()
        for a, b in patches:
            assert s.count(a) >= 1, (name, a[:40])
            i = s.rfind(a)  # the staged kernel follows the generic one
            s = s[:i] + b + s[i + len(a):]
        open(p, "w").write(s)
        for f in os.listdir(os.path.join(d, "csrc")):
            fp = os.path.join(d, "csrc", f)
            if os.path.isfile(fp) and (f.endswith((".h", ".hip", ".cpp")) or f == "Makefile"):
                t = open(fp).read().replace('../../include/', '../include/')
                open(fp, "w").write(t)
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(d, "csrc"), "OUT=" + os.path.join(d, "out")])
        print("built", name)


def run():
    sys.path.insert(0, ROOT)
    from kueue_oss_amd import native, synth
    snap_doc, wls = synth.config_c3(n_workloads=1024)
    res = {}
    for name in VARIANTS:
        so = os.path.join(EXP, name, "out", "libkueue_tas.so")
        lib = ctypes.CDLL(so)  # a patched build: its build id differs from the tree's on purpose
        native._bind(lib)
        snap = native.TASFlavorSnapshot(snap_doc, lib=lib)
        snap.compile(wls)
        runs = []
        for _ in range(25):
            snap.run_compiled()
            runs.append(snap.last_stage_times())
        res[name] = {k: round(sorted(r[k] for r in runs)[len(runs) // 2], 4) for k in runs[0]}
        print(json.dumps({name: res[name]}), flush=True)
        del snap
    print(json.dumps(res))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
