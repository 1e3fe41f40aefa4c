"""Helpers to load the golden fixtures and compare result lists."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tas_find_topology_assignments.json")


def load_cases(scope_in=True):
    with open(GOLDEN) as f:
        doc = json.load(f)
    cases = doc["cases"]
    if scope_in:
        cases = [c for c in cases if c["scope"] == "in"]
    return cases


def diff_against_golden(case, results):
    """Compare [{"name","assignment","reason"}] with the case's expectations
    (TASAssignmentsResult equality of tas_cache_test.go:6332-6334)."""
    got = {r["name"]: r for r in results}
    want = {ps["name"]: ps for ps in case["podSets"]}
    problems = []
    if set(got) != set(want):
        problems.append(f"podset names differ: got {sorted(got)} want {sorted(want)}")
    for name, ps in want.items():
        g = got.get(name)
        if g is None:
            continue
        if g["reason"] != ps["wantReason"]:
            problems.append(f"{name}: reason {g['reason']!r} != {ps['wantReason']!r}")
        if g["assignment"] != ps["wantAssignment"]:
            problems.append(f"{name}: assignment {g['assignment']} != {ps['wantAssignment']}")
    return problems
