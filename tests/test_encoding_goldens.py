"""v1beta2 compact TopologyAssignment encoding (pkg/util/tas/tas_assignment.go
:135-259): the oracle's restatement against the reference's own vectors
(tas_assignment_test.go bothWaysTestCases / oneWayTestCases, transcribed by
tools/extract_encoding_goldens.py)."""
import json
import os

import pytest

import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "tas_v1beta2_encoding.json")))["cases"]


def test_fixture_inventory():
    assert len(CASES) == 12 and sum(c["bothWays"] for c in CASES) == 10


@pytest.mark.parametrize("case", [c for c in CASES if c["bothWays"]], ids=lambda c: f"L{c['line']}")
def test_oracle_v1beta2_from(case):
    assert oracle_lib.v1beta2_from(case["internal"]) == case["v1beta2"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"L{c['line']}")
def test_oracle_internal_from(case):
    got = oracle_lib.internal_from(case["v1beta2"])
    assert got == case["internal"]
    assert [d["count"] for d in got["domains"]] == case["podCounts"]
    assert len(got["domains"]) == case["totalDomainCount"]
