"""Writes tests/golden/snapshot_queries.json: the reference's own table tests
for the snapshot queries other callers make, transcribed case by case.

  has_level      pkg/cache/scheduler/tas_flavor_snapshot_test.go:362-428 (TestHasLevel)
  quantity       pkg/resources/requests_test.go:320-380 (TestResourceQuantityRoundTrips)
                 and the values of tas_flavor_snapshot_test.go:33-72
  free_capacity  pkg/cache/scheduler/tas_flavor_snapshot_test.go:33-72 (TestFreeCapacityPerDomain)
"""
import json
import os

GI = 1024 ** 3
SRC = "pkg/cache/scheduler/tas_flavor_snapshot_test.go"

has_level = {
    "source": SRC + ":362-428",
    "levels": ["level-1", "level-2"],
    "cases": [
        {"name": "topology request nil", "request": None, "want": False},
        {"name": "topology request empty", "request": {}, "want": False},
        {"name": "required", "request": {"required": "level-1"}, "want": True},
        {"name": "required - invalid level", "request": {"required": "invalid-level"}, "want": False},
        {"name": "preferred", "request": {"preferred": "level-1"}, "want": True},
        {"name": "preferred - invalid level", "request": {"preferred": "invalid-level"}, "want": False},
        {"name": "unconstrained", "request": {"unconstrained": True}, "want": True},
        {"name": "slice-only", "request": {"podSetSliceRequiredTopology": "level-1"}, "want": True},
        {"name": "slice-only - invalid level", "request": {"podSetSliceRequiredTopology": "invalid-level"},
         "want": False},
    ],
}

quantity = {
    "source": "pkg/resources/requests_test.go:320-380; " + SRC + ":33-72",
    "cases": [
        ["memory", 1, "1"], ["memory", 1000, "1k"], ["memory", 100000, "100k"], ["memory", 1000000, "1M"],
        ["memory", 1500000, "1500k"], ["memory", 1024, "1Ki"], ["memory", 128000, "125Ki"],
        ["memory", 1024 * 1024, "1Mi"], ["memory", 1536 * 1024, "1536Ki"], ["memory", GI, "1Gi"],
        ["memory", 10000000000, "9765625Ki"],
        # TestFreeCapacityPerDomain's values
        ["cpu", 1000, "1"], ["cpu", 2000, "2"], ["cpu", 500, "500m"], ["memory", 2 * GI, "2Gi"],
        ["memory", 4 * GI, "4Gi"], ["nvidia.com/gpu", 1, "1"],
    ],
}

free_capacity = {
    "source": SRC + ":33-72",
    # leafDomain state of the test: freeCapacity and tasUsage per domain
    "leaves": {
        "domain2": {"freeCapacity": {"cpu": 1000, "memory": 2 * GI},
                    "tasUsage": {"memory": 1 * GI, "cpu": 500}},
        "domain1": {"freeCapacity": {"memory": 4 * GI, "cpu": 2000, "nvidia.com/gpu": 1},
                    "tasUsage": {"cpu": 500, "nvidia.com/gpu": 1, "memory": 2 * GI}},
    },
    "expected": '{"domain1":{"freeCapacity":{"cpu":"2","memory":"4Gi","nvidia.com/gpu":"1"},"tasUsage":{"cpu":"500m",'
                '"memory":"2Gi","nvidia.com/gpu":"1"}},"domain2":{"freeCapacity":{"cpu":"1","memory":"2Gi"},'
                '"tasUsage":{"cpu":"500m","memory":"1Gi"}}}',
}

out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "snapshot_queries.json")
with open(out, "w") as f:
    json.dump({"has_level": has_level, "quantity": quantity, "free_capacity": free_capacity}, f, indent=1)
print(out)
