"""Node joins on a C3-shaped snapshot: the cost of one join and of a batch of
64 joins (new hosts under existing racks) through kueue_tas_host_update_nodes,
and whether the device took them by splice or by reload.

usage: python tools/probe_join.py [--emu] [--shape 4,16,64,32] [--reps 3]
  --emu: the CPU SIMT emulator build (tests/emu), for host-side timing here
"""
import argparse
import copy
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kueue_oss_amd import TASFlavorSnapshot, native, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--emu", action="store_true")
    ap.add_argument("--shape", default="4,16,64,32")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    lib = None
    if a.emu:
        lib = native.load_library(os.path.join(ROOT, "tests", "emu", "_build", "libkueue_tas_emu.so"))
    shape = tuple(int(x) for x in a.shape.split(","))
    doc, wls = synth.config_c3(n_workloads=64, shape=shape)
    snap = TASFlavorSnapshot(doc, lib=lib) if lib else TASFlavorSnapshot(doc)
    snap.compile(wls)
    snap.run_compiled()
    N = len(doc["nodes"])
    host = "kubernetes.io/hostname"
    k = 0
    for rep in range(a.reps):
        joins = []
        for _ in range(65):
            nd = copy.deepcopy(doc["nodes"][k * 983 % N])
            nd["name"] = f"{nd['name']}-join{k}"
            nd["labels"][host] = f"{nd['labels'][host]}-join{k}"
            joins.append(nd)
            k += 1
        c0 = snap.snapshot_counters()
        t0 = time.perf_counter()
        r1 = snap.update_nodes(joins[:1])
        t1 = time.perf_counter()
        print(f"  join1 detail {snap.last_update_detail()}", flush=True)
        t1 = time.perf_counter()
        r64 = snap.update_nodes(joins[1:])
        t2 = time.perf_counter()
        c1 = snap.snapshot_counters()
        snap.run_compiled()
        t3 = time.perf_counter()
        d64 = snap.last_update_detail()
        print(f"rep {rep}: join1 {1e3 * (t1 - t0):.3f} ms  join64 {1e3 * (t2 - t1):.3f} ms  "
              f"next batch {1e3 * (t3 - t2):.3f} ms  rebuilt {r1 or r64}  loads/splices {c0} -> {c1}\n  join64 detail {d64}", flush=True)
    snap.close()


if __name__ == "__main__":
    main()
