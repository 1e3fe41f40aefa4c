"""The CPU oracle reproduces every in-scope golden case transcribed from the
reference's TestFindTopologyAssignments (pkg/cache/scheduler/tas_cache_test.go)."""
import pytest

import oracle_lib
from golden_util import diff_against_golden, load_cases

CASES = load_cases()


def test_fixture_inventory():
    from golden_util import load_cases as lc
    allc = lc(scope_in=False)
    assert len(allc) == 104  # 104 named cases in the reference table (:383-6266)
    # every case in scope: incl. the 4 elastic workload-slice cases (:5524-5733)
    # and the 18 TASBalancedPlacement cases (:2437-3884)
    assert len(CASES) == 104
    assert sum(1 for c in CASES if c.get("featureGates", {}).get("TASBalancedPlacement")) == 18


@pytest.mark.parametrize("case", CASES, ids=[f"L{c['line']}" for c in CASES])
def test_oracle_matches_golden(case):
    res = oracle_lib.run_case(case)["results"]
    assert diff_against_golden(case, res) == []
