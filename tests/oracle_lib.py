"""ctypes loader for the CPU oracle (oracle/_build/libtas_oracle.so).

Test infrastructure: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libtas_oracle.so")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    lib = ctypes.CDLL(ORACLE_SO)
    lib.tas_oracle_run_case.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    lib.tas_oracle_run_case.restype = ctypes.c_int
    lib.tas_oracle_eval_workloads.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_void_p)]
    lib.tas_oracle_eval_workloads.restype = ctypes.c_int
    lib.tas_oracle_session.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    lib.tas_oracle_session.restype = ctypes.c_int
    lib.tas_oracle_encoding.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.tas_oracle_encoding.restype = ctypes.c_int
    lib.tas_oracle_free.argtypes = [ctypes.c_void_p]
    _lib = lib
    return lib


def _take(lib, p):
    s = ctypes.cast(p, ctypes.c_char_p).value.decode()
    lib.tas_oracle_free(p)
    return json.loads(s)


def run_case(case: dict) -> dict:
    """Returns {"results": [...]} or raises on oracle error."""
    lib = load()
    out = ctypes.c_void_p()
    rc = lib.tas_oracle_run_case(json.dumps(case).encode(), ctypes.byref(out))
    doc = _take(lib, out)
    if rc != 0:
        raise RuntimeError(doc.get("error"))
    return doc


def eval_workloads(snapshot_case: dict, workloads: list, threads: int = 1, emit: bool = True):
    """Evaluates each workload independently; returns (results, seconds)."""
    lib = load()
    out = ctypes.c_void_p()
    secs = ctypes.c_double()
    rc = lib.tas_oracle_eval_workloads(json.dumps(snapshot_case).encode(),
                                       json.dumps({"workloads": workloads}).encode(),
                                       threads, 1 if emit else 0, ctypes.byref(secs), ctypes.byref(out))
    doc = _take(lib, out)
    if rc != 0:
        raise RuntimeError(doc.get("error"))
    return doc["results"], secs.value


def session(snapshot_case: dict, ops: list) -> list:
    """Applies find / fits / add / remove ops in order on one snapshot; one result per op."""
    lib = load()
    out = ctypes.c_void_p()
    rc = lib.tas_oracle_session(json.dumps(snapshot_case).encode(), json.dumps({"ops": ops}).encode(),
                                ctypes.byref(out))
    doc = _take(lib, out)
    if rc != 0:
        raise RuntimeError(doc.get("error"))
    return doc["results"]


def _encoding(doc: dict, direction: int) -> dict:
    lib = load()
    out = ctypes.c_void_p()
    rc = lib.tas_oracle_encoding(json.dumps(doc).encode(), direction, ctypes.byref(out))
    res = _take(lib, out)
    if rc != 0:
        raise RuntimeError(res.get("error"))
    return res


def v1beta2_from(internal: dict) -> dict:
    """V1Beta2From (pkg/util/tas/tas_assignment.go:251-259)."""
    return _encoding(internal, 0)


def internal_from(v1beta2: dict) -> dict:
    """InternalFrom (pkg/util/tas/tas_assignment.go:124-133)."""
    return _encoding(v1beta2, 1)


def preemption_search(snapshot_case: dict, setup: list, podsets: list, candidates: list) -> dict:
    """Oracle restatement of the TAS part of preemption's `minimal`
    (pkg/scheduler/preemption/preemption.go:307-345, workloadFits :614-625
    reduced to FindTopologyAssignmentsForWorkload(...).Failure() == nil):
    candidates are removed one by one (snapshot.RemoveWorkload ->
    RemoveUsage -> updateTASUsage on the oracle snapshot) and the workload is
    re-evaluated after each; on the first fit, fillBackWorkloads adds the
    targets back in reverse order with the reference's swap-delete.  Every
    evaluation replays `setup` (ops that put the candidates' usage in) on a
    fresh oracle snapshot.  Evaluates every prefix, like the device batch."""
    def fits(removed):
        ops = list(setup) + [{"op": "remove", "usage": candidates[c]} for c in removed]
        ops.append({"op": "find", "podSets": podsets})
        res = session(snapshot_case, ops)[-1]
        return all(not r["reason"] for r in res)

    pfits = [fits(list(range(i + 1))) for i in range(len(candidates))]
    first = next((i for i, f in enumerate(pfits) if f), -1)
    targets = None
    fill = 0
    if first >= 0:
        targets = list(range(first + 1))
        for i in range(len(targets) - 2, -1, -1):
            fill += 1
            if fits([t for j, t in enumerate(targets) if j != i]):
                targets[i] = targets[-1]
                targets.pop()
    return {"prefixFits": pfits, "firstFit": first, "targets": targets, "fillBackEvals": fill}
