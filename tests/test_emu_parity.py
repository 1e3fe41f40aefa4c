"""Kernel logic on CPU: the unmodified HIP sources compiled against the
test-only SIMT emulator (tests/emu) must match the golden fixtures and the
oracle.  This is not the product path (that is tests/test_gpu_parity.py on an
MI355X); it checks the wave-level algorithm where no GPU is available."""
import os
import random
import subprocess

import pytest

import oracle_lib
from golden_util import diff_against_golden, load_cases
from kueue_oss_amd import TASFlavorSnapshot, native, synth

HERE = os.path.dirname(os.path.abspath(__file__))
EMU_SO = os.path.join(HERE, "emu", "_build", "libkueue_tas_emu.so")


@pytest.mark.parametrize("list_cap", [0, 64])
def test_emulated_kernels_match_goldens(emu_lib, list_cap):
    bad = []
    for case in load_cases():
        snap = TASFlavorSnapshot(case, list_cap=list_cap, lib=emu_lib)
        res = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        if diff_against_golden(case, res):
            bad.append(case["line"])
    assert bad == []


@pytest.mark.parametrize("seed,list_cap,max_nodes,n", [(11, 0, 60, 250), (12, 64, 60, 250), (13, 64, 400, 60), (21, 128, 600, 60)])
def test_emulated_kernels_match_oracle_random(emu_lib, seed, list_cap, max_nodes, n):
    rng = random.Random(seed)
    for i in range(n):
        case = synth.random_case(rng, max_nodes=max_nodes)
        want = oracle_lib.run_case(case)["results"]
        snap = TASFlavorSnapshot(case, list_cap=list_cap, lib=emu_lib)
        got = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert got == want, (i, got, want)


@pytest.mark.parametrize("list_cap,n", [(64, 24), (128, 40)])
def test_emulated_kernels_match_oracle_c3_small(emu_lib, list_cap, n):
    # list_cap 128: descents longer than the LDS take the histogram threshold walk
    snap_doc, wls = synth.config_c3(n_workloads=n, shape=(2, 4, 16, 32))
    want, _ = oracle_lib.eval_workloads(snap_doc, wls)
    snap = TASFlavorSnapshot(snap_doc, list_cap=list_cap, lib=emu_lib)
    got = snap.find_topology_assignments_for_workloads(wls)
    snap.close()
    assert got == want


@pytest.mark.parametrize("seed,big", [(31, True), (32, False)])
def test_emulated_fast_lfc_stress(emu_lib, seed, big):
    # fast LeastFreeCapacity leaf path: several histogram chunks, overflow values, all outcomes
    snap_doc, wls = synth.lfc_stress_case(random.Random(seed), n_nodes=4500, n_workloads=24, big=big)
    want, _ = oracle_lib.eval_workloads(snap_doc, wls)
    snap = TASFlavorSnapshot(snap_doc, lib=emu_lib)
    got = snap.find_topology_assignments_for_workloads(wls)
    snap.close()
    mism = [i for i in range(len(wls)) if got[i] != want[i]]
    assert mism == [], (mism[:5], wls[mism[0]][0]["count"] if mism else None)


def test_emulated_kernels_match_oracle_c4_jobset(emu_lib):
    # leader/worker groups with slice topology on a uniform fan-out tree (fused parent roll-up in fill)
    snap_doc, wls = synth.config_c4(n_workloads=16, shape=(2, 2, 8, 16))
    want, _ = oracle_lib.eval_workloads(snap_doc, wls)
    snap = TASFlavorSnapshot(snap_doc, list_cap=64, lib=emu_lib)
    got = snap.find_topology_assignments_for_workloads(wls)
    snap.close()
    mism = [i for i in range(len(wls)) if got[i] != want[i]]
    assert mism == [], (mism[:5], got[mism[0]] if mism else None, want[mism[0]] if mism else None)


@pytest.mark.parametrize("seed", [41, 42])
def test_emulated_int64_arithmetic_stress(emu_lib, seed):
    # Go int64 wrap, truncating division by huge / odd divisors, int32 truncation and clamp
    rng = random.Random(seed)
    for i in range(150):
        case = synth.arith_stress_case(rng)
        want = oracle_lib.run_case(case)["results"]
        snap = TASFlavorSnapshot(case, lib=emu_lib)
        got = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert got == want, (i, got, want)


def test_emulated_split_stats_path_matches_oracle(emu_lib):
    # KUEUE_TAS_CFG_SPLIT_STATS: the one-leaf staged fill with the ExclusionStats
    # counted by the concurrent fill_exclusion_kernel branch (the default counts them in the fill)
    rng = random.Random(14)
    for i in range(120):
        case = synth.random_case(rng)
        want = oracle_lib.run_case(case)["results"]
        snap = TASFlavorSnapshot(case, lib=emu_lib, split_stats=True, pair_fill=False)
        got = snap.find_topology_assignments_for_flavor(case["podSets"])
        snap.close()
        assert got == want, (i, got, want)


def test_emulated_two_resident_flavors_interleaved(emu_lib):
    # alternating batches of two resident contexts share the device's select
    # descriptor, re-uploaded only when the context changes
    doc_a, wls_a = synth.config_c3(n_workloads=8, shape=(2, 2, 8, 16))
    doc_b, wls_b = synth.config_c4(n_workloads=4, shape=(2, 2, 4, 16))
    want_a, _ = oracle_lib.eval_workloads(doc_a, wls_a)
    want_b, _ = oracle_lib.eval_workloads(doc_b, wls_b)
    a = TASFlavorSnapshot(doc_a, lib=emu_lib)
    b = TASFlavorSnapshot(doc_b, lib=emu_lib)
    for _ in range(2):
        assert a.find_topology_assignments_for_workloads(wls_a) == want_a
        assert b.find_topology_assignments_for_workloads(wls_b) == want_b
    a.close()
    b.close()


def _class_collide(make):
    """The speculative merge of the host parts' phase-1 classes (equal 64-bit
    hashes taken as equal, verified exactly while the device runs) with every
    hash forced equal (KUEUE_TAS_CFG_CLASS_COLLIDE): the verification fails,
    the chunk re-runs with the exact merge, and every result is the oracle's."""
    doc, wls = synth.config_c2(n_workloads=96, shape=(2, 2, 4, 8))
    snap = make(doc)
    snap.compile(wls)
    snap.run_compiled(flags=TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES)
    got = snap.last_results()
    reruns = snap.merge_reruns()
    snap.close()
    want, _ = oracle_lib.eval_workloads(doc, wls, threads=4)
    assert got == want
    assert reruns >= 1


def test_emulated_class_collide(emu_lib):  # noqa: F811
    _class_collide(lambda d: TASFlavorSnapshot(d, lib=emu_lib, class_collide=True))


@pytest.mark.gpu
def test_class_collide_on_gpu():
    _class_collide(lambda d: TASFlavorSnapshot(d, class_collide=True))
