"""Elastic workload slices (ElasticJobsViaWorkloadSlicesWithTAS):
FindTopologyAssignmentsForFlavor places only the delta of a workers PodSet
that carries a PreviousAssignment (tas_elastic_workloads.go:35-127: scale
up keeps the previous pods and assumes their usage, scale down truncates,
same count reuses; a stale previous assignment falls back to fresh
placement).  The reference's 4 cases (tas_cache_test.go:5524-5733) are in
the extracted goldens (tests/golden/tas_find_topology_assignments.json,
checked by test_oracle_goldens / test_emu_parity / test_gpu_parity); here
random cases: library == oracle, on the emulated library and the GPU."""
import json
import random

import pytest

import oracle_lib
from kueue_oss_amd import TASFlavorSnapshot, synth


def _random(make, seed, n):
    rng = random.Random(seed)
    run = lambda case: oracle_lib.run_case(case)["results"]  # noqa: E731
    kinds = set()
    for _ in range(n):
        c = synth.elastic_case(rng, run)
        want = run(c)
        snap = make({k: v for k, v in c.items() if k != "podSets"})
        got = snap.find_topology_assignments_for_flavor(c["podSets"])
        snap.close()
        assert got == want, json.dumps(c)
        for ps in c["podSets"]:
            if "previousAssignment" in ps:
                prev = sum(d["count"] for d in ps["previousAssignment"]["domains"])
                kinds.add("up" if ps["count"] > prev else "down" if ps["count"] < prev else "same")
    assert kinds == {"up", "down", "same"}


def test_emulated_random(emu_lib):
    _random(lambda d: TASFlavorSnapshot(d, lib=emu_lib), 21, 150)


@pytest.mark.gpu
def test_random_on_gpu():
    _random(lambda d: TASFlavorSnapshot(d), 22, 200)
