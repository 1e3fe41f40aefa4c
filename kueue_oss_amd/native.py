"""ctypes binding of libkueue_tas.so (include/kueue_tas.h).

This is the product path: every evaluation runs the HIP kernels of
``csrc/tas_kernels.hip``.  There is no CPU fallback — if the shared library or
a HIP device is missing, construction raises ``NativeLibraryMissing``.

``TASFlavorSnapshot`` mirrors the reference's Go type of the same name
(pkg/cache/scheduler/tas_flavor_snapshot.go:109-137) at the granularity the
host layer exposes: build from a snapshot document (nodes, pods, levels,
flavor node labels/tolerations, TAS usage, feature gates), then
``find_topology_assignments_for_flavor`` (:519) or the batched
``find_topology_assignments_for_workloads`` (the nominate batch of
pkg/scheduler/scheduler.go:583-619).
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

_PKG = os.path.dirname(os.path.abspath(__file__))
_CSRC = os.path.join(_PKG, "csrc")
_BUILD = os.path.join(_PKG, "_build")
_LIB = None


class NativeLibraryMissing(RuntimeError):
    """libkueue_tas.so could not be loaded or no HIP device is usable."""


def library_path() -> str:
    return os.path.join(_BUILD, "libkueue_tas.so")


def build_native(jobs: int = 4) -> str:
    """Compile libkueue_tas.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", _CSRC], check=True)
    return library_path()


class KueueTasConfig(ctypes.Structure):
    _fields_ = [("list_cap", ctypes.c_int32), ("max_batch", ctypes.c_int32),
                ("device", ctypes.c_int32), ("flags", ctypes.c_int32)]


EXPORTED_SYMBOLS = [
    "kueue_tas_abi_version", "kueue_tas_ctx_create", "kueue_tas_ctx_destroy", "kueue_tas_last_error",
    "kueue_tas_snapshot_load", "kueue_tas_snapshot_apply_deltas", "kueue_tas_eval_batch", "kueue_tas_fetch_entries",
    "kueue_tas_last_timings", "kueue_tas_last_stage_times", "kueue_tas_last_eval_ticks", "kueue_tas_last_host_times", "kueue_tas_last_entries", "kueue_tas_last_eval_profile", "kueue_tas_last_stats", "kueue_tas_last_fill_paths", "kueue_tas_last_counters", "kueue_tas_host_create", "kueue_tas_host_destroy",
    "kueue_tas_host_last_error", "kueue_tas_host_find", "kueue_tas_host_find_batch",
    "kueue_tas_host_compile", "kueue_tas_host_run_compiled", "kueue_tas_host_last_timings",
    "kueue_tas_host_last_stage_times", "kueue_tas_host_last_eval_ticks", "kueue_tas_host_last_device_host_times", "kueue_tas_host_last_eval_profile", "kueue_tas_host_last_profile", "kueue_tas_host_last_stats", "kueue_tas_free",
    "kueue_tas_fits", "kueue_tas_host_update_usage", "kueue_tas_host_fits", "kueue_tas_host_preemption_search", "kueue_tas_host_update_pods",
    "kueue_tas_snapshot_set_free", "kueue_tas_snapshot_set_leaf_attrs", "kueue_tas_host_update_nodes",
    "kueue_tas_encode_v1beta2", "kueue_tas_snapshot_load_names", "kueue_tas_encode_v1beta2_leaves",
    "kueue_tas_host_v1beta2_from", "kueue_tas_host_internal_from", "kueue_tas_host_find_v1beta2",
    "kueue_tas_host_v1beta2_last", "kueue_tas_host_last_results", "kueue_tas_admit", "kueue_tas_host_set_shard",
    "kueue_tas_host_last_assignments", "kueue_tas_host_admit", "kueue_tas_host_apply_deltas",
    "kueue_tas_host_last_deltas", "kueue_tas_host_run", "kueue_tas_build_id",
    "kueue_tas_host_has_level", "kueue_tas_host_assignment_stale", "kueue_tas_host_free_capacity_json",
    "kueue_tas_resource_quantity_string", "kueue_tas_host_ctx", "kueue_tas_host_leaf_ids",
    "kueue_tas_host_compile_workload", "kueue_tas_host_last_admit_times", "kueue_tas_last_admit_stats",
    "kueue_tas_host_last_admit_stats", "kueue_tas_host_find_workload",
    "kueue_tas_snapshot_set_leaf_live", "kueue_tas_snapshot_set_leaf_tags", "kueue_tas_last_entry_tags",
    "kueue_tas_host_last_host_detail", "kueue_tas_host_last_update_detail", "kueue_tas_eval_batch_ptrs", "kueue_tas_set_stage_timing",
    "kueue_tas_host_set_stage_timing", "kueue_tas_host_stage_accum", "kueue_tas_snapshot_splice", "kueue_tas_snapshot_counters",
    "kueue_tas_device_bytes",
    "kueue_tas_last_alias_fills", "kueue_tas_host_last_stats_ext", "kueue_tas_last_fill_profile",
    "kueue_tas_snapshot_usage_mark", "kueue_tas_snapshot_usage_changes", "kueue_tas_snapshot_apply_deltas_mirrored",
    "kueue_tas_host_partial_admission_search", "kueue_tas_last_host_trace", "kueue_tas_merge_reruns",
    "kueue_tas_select_groups", "kueue_tas_admit_table", "kueue_tas_admit_block", "kueue_tas_copy_to_host",
    "kueue_tas_host_admit_block",
]

# the Makefile's SRC_HASH inputs, in order
_HASHED_SOURCES = ("tas_device.hip", "tas_host.cpp", "tas_internal.h", "tas_kernels.hip", "json_reader.h",
                   "label_selectors.h", "tas_balanced.h", "tas_pool.h", os.path.join("..", "..", "include", "kueue_tas.h"),
                   os.path.join("..", "..", "include", "kueue_tas_debug.h"))


def source_hash() -> str | None:
    """The build id a library built from this tree's sources reports (None when
    the sources are not shipped next to the package)."""
    import hashlib

    h = hashlib.sha256()
    for f in _HASHED_SOURCES:
        p = os.path.join(_CSRC, f)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]

# kueue_tas_delta {int32 leaf, int32 col, int64 delta} as a numpy record
DELTA_DTYPE = [("leaf", "<i4"), ("col", "<i4"), ("delta", "<i8")]


def load_library(path: str | None = None):
    """Load the in-tree libkueue_tas.so (raises NativeLibraryMissing).

    ``path`` loads another build of the same C-ABI instead (tests use the
    CPU-emulated build of tests/emu to check kernel logic without a GPU)."""
    global _LIB
    if path is None and _LIB is not None:
        return _LIB
    p = path or library_path()
    if not os.path.exists(p):
        raise NativeLibraryMissing(f"{p} not built (run __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:  # pragma: no cover - environment specific
        raise NativeLibraryMissing(str(e)) from e
    _bind(lib)
    if path is None:
        want = source_hash()
        got = lib.kueue_tas_build_id().decode()
        if want is not None and got != want:
            raise NativeLibraryMissing(f"{p} was built from other sources (build id {got}, tree {want}): "
                                       "run __graft_entry__.build()")
        _LIB = lib
    return lib


def _bind(lib):
    c = ctypes
    lib.kueue_tas_abi_version.restype = c.c_int
    lib.kueue_tas_build_id.restype = c.c_char_p
    lib.kueue_tas_host_create.argtypes = [c.c_char_p, c.POINTER(KueueTasConfig)]
    lib.kueue_tas_host_create.restype = c.c_void_p
    lib.kueue_tas_host_destroy.argtypes = [c.c_void_p]
    lib.kueue_tas_host_last_error.argtypes = [c.c_void_p]
    lib.kueue_tas_host_last_error.restype = c.c_char_p
    lib.kueue_tas_host_find.argtypes = [c.c_void_p, c.c_char_p, c.c_int32, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_find.restype = c.c_int
    lib.kueue_tas_host_find_batch.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_find_batch.restype = c.c_int
    lib.kueue_tas_host_compile.argtypes = [c.c_void_p, c.c_char_p]
    lib.kueue_tas_host_compile.restype = c.c_int
    lib.kueue_tas_host_run_compiled.argtypes = [c.c_void_p, c.POINTER(c.c_uint64)]
    lib.kueue_tas_host_run_compiled.restype = c.c_int
    lib.kueue_tas_host_run.argtypes = [c.c_void_p, c.c_uint32, c.POINTER(c.c_uint64)]
    lib.kueue_tas_host_run.restype = c.c_int
    lib.kueue_tas_host_last_timings.argtypes = [c.c_void_p, c.POINTER(c.c_float), c.POINTER(c.c_int64)]
    lib.kueue_tas_host_last_stage_times.argtypes = [c.c_void_p, c.POINTER(c.c_float), c.c_int]
    lib.kueue_tas_host_last_eval_profile.argtypes = [c.c_void_p, c.POINTER(c.c_int32), c.c_size_t]
    lib.kueue_tas_host_last_device_host_times.argtypes = [c.c_void_p, c.POINTER(c.c_double), c.c_int]
    lib.kueue_tas_host_last_eval_ticks.argtypes = [c.c_void_p, c.POINTER(c.c_int32), c.c_size_t]
    lib.kueue_tas_host_last_profile.argtypes = [c.c_void_p, c.POINTER(c.c_double)]
    lib.kueue_tas_host_last_host_detail.argtypes = [c.c_void_p, c.POINTER(c.c_double), c.c_int]
    lib.kueue_tas_host_last_update_detail.argtypes = [c.c_void_p, c.POINTER(c.c_double), c.c_int]
    lib.kueue_tas_host_set_stage_timing.argtypes = [c.c_void_p, c.c_int32]
    lib.kueue_tas_snapshot_counters.argtypes = [c.c_void_p, c.POINTER(c.c_int64), c.POINTER(c.c_int64)]
    lib.kueue_tas_device_bytes.argtypes = [c.c_void_p, c.POINTER(c.c_int64), c.POINTER(c.c_int64)]
    lib.kueue_tas_select_groups.argtypes = [c.c_void_p, c.POINTER(c.c_int64), c.POINTER(c.c_int64)]
    lib.kueue_tas_host_stage_accum.argtypes = [c.c_void_p, c.POINTER(c.c_float), c.c_int, c.POINTER(c.c_int64),
                                               c.POINTER(c.c_int64), c.c_int32]
    lib.kueue_tas_host_last_admit_times.argtypes = [c.c_void_p, c.POINTER(c.c_double)]
    lib.kueue_tas_last_admit_stats.argtypes = [c.c_void_p, c.POINTER(c.c_int64)]
    lib.kueue_tas_host_last_admit_stats.argtypes = [c.c_void_p, c.POINTER(c.c_int64)]
    lib.kueue_tas_host_find_workload.argtypes = [c.c_void_p, c.c_char_p, c.c_int32, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_find_workload.restype = c.c_int
    lib.kueue_tas_host_last_stats.argtypes = [c.c_void_p, c.POINTER(c.c_int64)]
    lib.kueue_tas_host_last_stats_ext.argtypes = [c.c_void_p, c.POINTER(c.c_int64), c.c_int32]
    lib.kueue_tas_last_alias_fills.argtypes = [c.c_void_p]
    lib.kueue_tas_last_alias_fills.restype = c.c_int64
    lib.kueue_tas_last_fill_profile.argtypes = [c.c_void_p, c.POINTER(c.c_int32), c.c_size_t]
    lib.kueue_tas_last_fill_profile.restype = c.c_int64
    lib.kueue_tas_host_update_usage.argtypes = [c.c_void_p, c.c_char_p, c.c_int32]
    lib.kueue_tas_host_update_usage.restype = c.c_int
    lib.kueue_tas_host_fits.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_int32)]
    lib.kueue_tas_host_fits.restype = c.c_int
    for name in ("kueue_tas_host_v1beta2_from", "kueue_tas_host_internal_from"):
        getattr(lib, name).argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_void_p)]
        getattr(lib, name).restype = c.c_int
    lib.kueue_tas_host_find_v1beta2.argtypes = [c.c_void_p, c.c_char_p, c.c_int32, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_find_v1beta2.restype = c.c_int
    lib.kueue_tas_host_v1beta2_last.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_last_results.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_set_shard.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    lib.kueue_tas_host_set_shard.restype = c.c_int
    lib.kueue_tas_host_last_assignments.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t)]
    lib.kueue_tas_host_last_assignments.restype = c.c_int
    lib.kueue_tas_host_admit.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t,
                                         c.POINTER(c.c_size_t), c.POINTER(c.c_size_t)]
    lib.kueue_tas_host_last_deltas.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    lib.kueue_tas_host_admit_block.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_int32, c.c_void_p,
                                               c.c_size_t, c.POINTER(c.c_size_t), c.POINTER(c.c_size_t)]
    lib.kueue_tas_host_admit_block.restype = c.c_int
    lib.kueue_tas_host_last_deltas.restype = c.c_int
    lib.kueue_tas_host_admit.restype = c.c_int
    lib.kueue_tas_host_apply_deltas.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    lib.kueue_tas_host_apply_deltas.restype = c.c_int
    lib.kueue_tas_host_last_results.restype = c.c_int
    lib.kueue_tas_host_v1beta2_last.restype = c.c_int
    lib.kueue_tas_host_preemption_search.argtypes = [c.c_void_p, c.c_char_p, c.c_char_p, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_preemption_search.restype = c.c_int
    lib.kueue_tas_host_partial_admission_search.argtypes = [c.c_void_p, c.c_char_p, c.c_int32, c.c_int32,
                                                            c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_partial_admission_search.restype = c.c_int
    lib.kueue_tas_host_update_nodes.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_int32)]
    lib.kueue_tas_host_update_nodes.restype = c.c_int
    lib.kueue_tas_host_update_pods.argtypes = [c.c_void_p, c.c_char_p]
    lib.kueue_tas_host_update_pods.restype = c.c_int
    lib.kueue_tas_free.argtypes = [c.c_void_p]
    lib.kueue_tas_host_has_level.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_int32)]
    lib.kueue_tas_host_has_level.restype = c.c_int
    lib.kueue_tas_host_assignment_stale.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_int32), c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_assignment_stale.restype = c.c_int
    lib.kueue_tas_host_free_capacity_json.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_free_capacity_json.restype = c.c_int
    lib.kueue_tas_resource_quantity_string.argtypes = [c.c_char_p, c.c_int64, c.c_char_p, c.c_size_t,
                                                       c.POINTER(c.c_size_t)]
    lib.kueue_tas_resource_quantity_string.restype = c.c_int
    lib.kueue_tas_host_ctx.argtypes = [c.c_void_p]
    lib.kueue_tas_host_ctx.restype = c.c_void_p
    lib.kueue_tas_host_leaf_ids.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_leaf_ids.restype = c.c_int
    lib.kueue_tas_host_compile_workload.argtypes = [c.c_void_p, c.c_char_p, c.c_int32,
                                                    c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t),
                                                    c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t), c.POINTER(c.c_int32),
                                                    c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t),
                                                    c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t),
                                                    c.POINTER(c.c_void_p)]
    lib.kueue_tas_host_compile_workload.restype = c.c_int


def resource_quantity_string(name: str, value: int, lib=None) -> str:
    """resources.ResourceQuantityString (pkg/resources/requests.go:147) via the library."""
    lib = lib if lib is not None else load_library()
    buf = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t()
    if lib.kueue_tas_resource_quantity_string(name.encode(), value, buf, 64, ctypes.byref(n)):
        raise RuntimeError("kueue_tas_resource_quantity_string failed")
    return buf.value.decode()


def _take(lib, p) -> dict:
    s = ctypes.cast(p, ctypes.c_char_p).value.decode()
    lib.kueue_tas_free(p)
    return json.loads(s)


class TASFlavorSnapshot:
    """Device-resident TAS snapshot of one ResourceFlavor (reference
    tas_flavor_snapshot.go:109).  ``snapshot`` follows the fixture schema of
    tools/extract_goldens.py (podSets ignored)."""

    def __init__(self, snapshot: dict, list_cap: int = 0, max_batch: int = 0, device: int = 0, lib=None,
                 packed_entries: bool = False, inline_stats: bool = False,
                 pair_fill: bool = True, serial_admit: bool = False, split_stats: bool = False,
                 fused_top: bool = False, host_values: bool = False, category_fill: bool = True,
                 class_collide: bool = False, lfc_in_fill: bool = False):
        self._lib = lib if lib is not None else load_library()
        cfg = KueueTasConfig(list_cap, max_batch, device, (1 if packed_entries else 0) | (2 if inline_stats else 0)
                              | (0 if pair_fill else 4) | (8 if serial_admit else 0) | (16 if split_stats else 0)
                              | (32 if fused_top else 0) | (64 if host_values else 0)
                              | (0 if category_fill else 128) | (256 if class_collide else 0)
                              | (512 if lfc_in_fill else 0))
        doc = {k: v for k, v in snapshot.items() if k != "podSets"}
        h = self._lib.kueue_tas_host_create(json.dumps(doc).encode(), ctypes.byref(cfg))
        if not h:
            raise NativeLibraryMissing("kueue_tas_host_create returned NULL")
        err = self._lib.kueue_tas_host_last_error(h).decode()
        if err:
            self._lib.kueue_tas_host_destroy(h)
            raise NativeLibraryMissing(err)
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.kueue_tas_host_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _err(self):
        return self._lib.kueue_tas_host_last_error(self._h).decode()

    def find_topology_assignments_for_flavor(self, podsets: list, simulate_empty: bool = False) -> list:
        """FindTopologyAssignmentsForFlavor (:519-594) for one workload's
        PodSets; returns [{"name", "assignment", "reason"}] in result order."""
        out = ctypes.c_void_p()
        rc = self._lib.kueue_tas_host_find(self._h, json.dumps(podsets).encode(), 1 if simulate_empty else 0,
                                           ctypes.byref(out))
        if rc != 0:
            raise RuntimeError(f"kueue_tas_host_find failed ({rc}): {self._err()}")
        return _take(self._lib, out)["results"]

    # ---- snapshot usage and the admission re-check (records: workload.TopologyDomainRequests,
    # [{"values": [...], "singlePodRequests": {...}, "count": n}]) ----
    def add_usage(self, records: list):
        """ClusterQueueSnapshot.AddUsage -> updateTASUsage (clusterqueue_snapshot.go:94-119)."""
        if self._lib.kueue_tas_host_update_usage(self._h, json.dumps(records).encode(), 1):
            raise RuntimeError(self._err())

    def remove_usage(self, records: list):
        """ClusterQueueSnapshot.RemoveUsage -> updateTASUsage (clusterqueue_snapshot.go:100-119)."""
        if self._lib.kueue_tas_host_update_usage(self._h, json.dumps(records).encode(), 0):
            raise RuntimeError(self._err())

    def update_nodes(self, nodes: list) -> bool:
        """Node events (nodesCache.sync, tas_nodes_cache.go:38-72): in place when the
        nodes keep their topology position and existing taint profiles / label values,
        else a rebuild.  Returns True when the snapshot was rebuilt."""
        r = ctypes.c_int32()
        if self._lib.kueue_tas_host_update_nodes(self._h, json.dumps(nodes).encode(), ctypes.byref(r)):
            raise RuntimeError(self._err())
        return bool(r.value)

    def update_pods(self, pods: list):
        """Non-TAS pod events (nonTasUsageCache.update/delete, tas_non_tas_pod_cache.go:46-116)
        applied to the resident snapshot: touched leaves recomputed and replaced on the device."""
        if self._lib.kueue_tas_host_update_pods(self._h, json.dumps(pods).encode()):
            raise RuntimeError(self._err())

    def fits(self, records: list) -> bool:
        """TASFlavorSnapshot.Fits (tas_flavor_snapshot.go:401-415), evaluated on the device."""
        f = ctypes.c_int32()
        if self._lib.kueue_tas_host_fits(self._h, json.dumps(records).encode(), ctypes.byref(f)):
            raise RuntimeError(self._err())
        return bool(f.value)

    def preemption_search(self, podsets: list, candidates: list) -> dict:
        """TAS part of preemption's `minimal` (pkg/scheduler/preemption/
        preemption.go:307-345): every candidate prefix evaluated in one device
        batch under a removal overlay, then fillBackWorkloads.  ``candidates``
        is a list of usage-record lists (the candidates' admitted usage), or
        that list already JSON-encoded (bytes)."""
        enc = candidates if isinstance(candidates, bytes) else json.dumps(candidates).encode()
        return self._json_call(self._lib.kueue_tas_host_preemption_search, podsets, enc)

    def partial_admission_search(self, podsets: list, simulate_empty: bool = False, max_batch: int = 0) -> dict:
        """PodSetReducer.Search (pkg/scheduler/flavorassigner/podset_reducer.go:37-86)
        over the TAS fit: PodSets carry ``count`` and optional ``minCount``
        (and ``tas: False`` for a PodSet outside TAS); sort.Search's decision
        tree is evaluated ``max_batch`` probes per device batch (0: 1023)."""
        return self._json_call(self._lib.kueue_tas_host_partial_admission_search, podsets,
                               1 if simulate_empty else 0, int(max_batch))

    # ---- v1beta2 wire format (pkg/util/tas/tas_assignment.go) ----
    def _json_call(self, fn, payload, *extra):
        out = ctypes.c_void_p()
        rc = fn(self._h, json.dumps(payload).encode(), *extra, ctypes.byref(out))
        if rc != 0:
            raise RuntimeError(f"{fn.__name__} failed ({rc}): {self._err()}")
        return _take(self._lib, out)

    def v1beta2_from(self, assignments: list) -> list:
        """V1Beta2From (tas_assignment.go:251-259) of internal assignments (None allowed), on the device."""
        return self._json_call(self._lib.kueue_tas_host_v1beta2_from, assignments)

    def internal_from(self, assignments: list) -> list:
        """InternalFrom (tas_assignment.go:124-133) of v1beta2 assignments."""
        return self._json_call(self._lib.kueue_tas_host_internal_from, assignments)

    def find_topology_assignments_v1beta2(self, podsets: list, simulate_empty: bool = False) -> list:
        """find_topology_assignments_for_flavor with the assignment in the v1beta2
        form ("topologyAssignment"), encoded on the device from the resident names."""
        return self._json_call(self._lib.kueue_tas_host_find_v1beta2, podsets, 1 if simulate_empty else 0)["results"]

    def last_v1beta2(self, materialize: bool = True):
        """v1beta2 form of every result of the last run_compiled ([[...] per workload])."""
        if not materialize:
            if self._lib.kueue_tas_host_v1beta2_last(self._h, None):
                raise RuntimeError(self._err())
            return None
        out = ctypes.c_void_p()
        if self._lib.kueue_tas_host_v1beta2_last(self._h, ctypes.byref(out)):
            raise RuntimeError(self._err())
        return _take(self._lib, out)

    def find_topology_assignments_for_workloads(self, workloads: list) -> list:
        """Evaluate many workloads independently against this snapshot in one
        device batch (Scheduler.nominate, scheduler.go:583-619)."""
        out = ctypes.c_void_p()
        rc = self._lib.kueue_tas_host_find_batch(self._h, json.dumps({"workloads": workloads}).encode(),
                                                 ctypes.byref(out))
        if rc != 0:
            raise RuntimeError(f"kueue_tas_host_find_batch failed ({rc}): {self._err()}")
        return _take(self._lib, out)["results"]

    def compile(self, workloads: list):
        rc = self._lib.kueue_tas_host_compile(self._h, json.dumps({"workloads": workloads}).encode())
        if rc != 0:
            raise RuntimeError(f"kueue_tas_host_compile failed ({rc}): {self._err()}")
        self._n_compiled = len(workloads)

    def last_timings(self):
        """(fill_ms, rollup_ms, select_ms, total_ms), (batches, evals, leader_evals) of the last run."""
        ms = (ctypes.c_float * 4)()
        cnt = (ctypes.c_int64 * 3)()
        self._lib.kueue_tas_host_last_timings(self._h, ms, cnt)
        return tuple(ms), tuple(cnt)

    def last_stats(self):
        """Work counters of the last run: dict(batches, evals, leader_evals,
        fill_evals, leaf_partial_evals, fill_launches, staged_cols, fill_paths:
        OR of the KUEUE_TAS_PATH_* bits of include/kueue_tas_debug.h,
        alias_fills: fill rows whose sliceState aliases state)."""
        st = (ctypes.c_int64 * 9)()
        self._lib.kueue_tas_host_last_stats_ext(self._h, st, 9)
        keys = ("batches", "evals", "leader_evals", "fill_evals", "leaf_partial_evals", "fill_launches", "staged_cols",
                "fill_paths", "alias_fills")
        return dict(zip(keys, list(st)))

    STAGES = ("fill", "rollup", "replicate", "lfc_branch", "select", "join_wait", "device_total")

    def last_stage_times(self):
        """Device ms per stage of the last run (HIP events; lfc_branch runs on the second stream concurrently with rollup..select), dict keyed by STAGES."""
        ms = (ctypes.c_float * len(self.STAGES))()
        self._lib.kueue_tas_host_last_stage_times(self._h, ms, len(self.STAGES))
        return dict(zip(self.STAGES, list(ms)))

    def last_eval_ticks(self, n: int):
        """Per-eval select-kernel time (100 MHz ticks) of the last device batch
        (diagnostics): [(total, findLevelWithFitDomains part)] * n."""
        buf = (ctypes.c_int32 * (2 * n))()
        self._lib.kueue_tas_host_last_eval_ticks(self._h, buf, n)
        return [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]

    PROF = ("lds_sort", "threshold_walk", "gather", "emit", "walk_sorted", "global_sort", "update_counts", "find_level",
            "tw_keys", "tw_select", "tw_emit", "setup", "final_leaf_walk",
            "fw_parents", "fw_children", "fw_loads", "fw_select", "fw_emit", "ws_filter", "sel_emit")

    def last_eval_profile(self, n: int):
        """Profiling build only: inclusive select-phase ticks per eval, dicts keyed by PROF."""
        k = len(self.PROF)
        buf = (ctypes.c_int32 * (k * n))()
        self._lib.kueue_tas_host_last_eval_profile(self._h, buf, n)
        return [dict(zip(self.PROF, buf[k * i: k * i + k])) for i in range(n)]

    DEVICE_HOST = ("compile", "classes", "enqueue", "wait", "pack_d2h", "copy_out", "compile_validate",
                   "compile_records")

    def last_device_host_times(self):
        """Host ms inside the device layer over the last run, dict keyed by DEVICE_HOST."""
        ms = (ctypes.c_double * 8)()
        self._lib.kueue_tas_host_last_device_host_times(self._h, ms, 8)
        return dict(zip(self.DEVICE_HOST, list(ms)))

    def last_profile(self):
        """Host wall ms of the last run_compiled: (staging, eval calls, decode, total)."""
        ms = (ctypes.c_double * 4)()
        self._lib.kueue_tas_host_last_profile(self._h, ms)
        return tuple(ms)

    HOST_DETAIL = ("groups", "compile", "build_pass", "values")

    def last_host_detail(self):
        """Finer host wall ms of the last run_compiled, dict keyed by HOST_DETAIL."""
        ms = (ctypes.c_double * 4)()
        self._lib.kueue_tas_host_last_host_detail(self._h, ms, 4)
        return dict(zip(self.HOST_DETAIL, list(ms)))

    UPDATE_DETAIL = ("parse", "events", "flush_joins", "splice_rows", "splice_device", "leaf_tags",
                     "evaluator_reset", "pushes", "total", "flush_mirror_fold", "flush_levels", "flush_leaf_arrays",
                     "flush_maps_ranks")

    def last_update_detail(self):
        """Host wall ms of the last update_nodes, dict keyed by UPDATE_DETAIL."""
        ms = (ctypes.c_double * 13)()
        self._lib.kueue_tas_host_last_update_detail(self._h, ms, 13)
        return {k: round(v, 3) for k, v in zip(self.UPDATE_DETAIL, list(ms))}

    def set_stage_timing(self, on: bool):
        """Record every device stage event (True, default) or only the fill bracket."""
        if self._lib.kueue_tas_host_set_stage_timing(self._h, 1 if on else 0):
            raise RuntimeError(self._err())

    def stage_accum(self, reset: bool = False):
        """Device stage ms summed over every run_compiled since the last reset:
        (dict keyed by STAGES, runs, fill launches)."""
        ms = (ctypes.c_float * len(self.STAGES))()
        runs, fills = ctypes.c_int64(), ctypes.c_int64()
        self._lib.kueue_tas_host_stage_accum(self._h, ms, len(self.STAGES), ctypes.byref(runs), ctypes.byref(fills),
                                             1 if reset else 0)
        return dict(zip(self.STAGES, list(ms))), runs.value, fills.value

    def snapshot_counters(self):
        """(snapshot loads, snapshot splices) of the device context so far."""
        lo, sp = ctypes.c_int64(), ctypes.c_int64()
        self._lib.kueue_tas_snapshot_counters(self.device_ctx(), ctypes.byref(lo), ctypes.byref(sp))
        return lo.value, sp.value

    def device_bytes(self):
        """(every device buffer, the per-batch evaluation state) of the device
        context, in bytes (kueue_tas_device_bytes)."""
        t, p2 = ctypes.c_int64(), ctypes.c_int64()
        self._lib.kueue_tas_device_bytes(self.device_ctx(), ctypes.byref(t), ctypes.byref(p2))
        return t.value, p2.value

    def last_results(self) -> list:
        """Results of the last run_compiled, one result list per compiled workload."""
        out = ctypes.c_void_p()
        if self._lib.kueue_tas_host_last_results(self._h, ctypes.byref(out)):
            raise RuntimeError(self._err())
        return _take(self._lib, out)["results"]

    # ---- data-parallel batches (kueue_tas.h "Data-parallel batches") ----
    def set_shard(self, ids):
        """run_compiled evaluates only the compiled workloads `ids` (global indices)."""
        import numpy as np
        a = np.ascontiguousarray(ids, dtype=np.int32)
        if self._lib.kueue_tas_host_set_shard(self._h, a.ctypes.data, a.size):
            raise RuntimeError(self._err())

    def last_assignments(self):
        """int32 quads of the last run_compiled: per workload (id, -1, failed, n)
        then (id, podset, leaf, count) per assigned domain."""
        import numpy as np
        n = ctypes.c_size_t()
        rc = self._lib.kueue_tas_host_last_assignments(self._h, None, 0, ctypes.byref(n))
        if rc not in (0, -5):
            raise RuntimeError(self._err())
        buf = np.empty(n.value, dtype=np.int32)
        if self._lib.kueue_tas_host_last_assignments(self._h, buf.ctypes.data, buf.size, ctypes.byref(n)):
            raise RuntimeError(self._err())
        return buf

    def admit(self, quads):
        """Admission (Fits + AddUsage, in workload order) over gathered quads on this
        replica; returns (admitted (id, 0/1) pairs [n, 2], deltas numpy DELTA_DTYPE)."""
        import numpy as np
        q = np.ascontiguousarray(quads, dtype=np.int32)
        # one header quad (id, -1, failed, n) per workload: the admitted
        # capacity without a sort (np.unique cost ~0.5 ms per 20k quads)
        heads = int(np.count_nonzero(q[1::4] < 0)) if q.size else 0
        adm = np.zeros((heads, 2), dtype=np.int32)
        nw = ctypes.c_size_t()
        nd = ctypes.c_size_t()
        rc = self._lib.kueue_tas_host_admit(self._h, q.ctypes.data, q.size, adm.ctypes.data, adm.size,
                                            ctypes.byref(nw), ctypes.byref(nd))
        if rc == -5 and nw.value > heads:  # workloads without a header quad: size by the library's count
            adm = np.zeros((nw.value, 2), dtype=np.int32)
            rc = self._lib.kueue_tas_host_admit(self._h, q.ctypes.data, q.size, adm.ctypes.data, adm.size,
                                                ctypes.byref(nw), ctypes.byref(nd))
        if rc:
            raise RuntimeError(self._err())
        deltas = np.zeros(nd.value, dtype=DELTA_DTYPE)
        if self._lib.kueue_tas_host_last_deltas(self._h, deltas.ctypes.data, deltas.size):
            raise RuntimeError(self._err())
        return adm[: nw.value], deltas

    def admit_block(self, block, lens, row_words=None):
        """admit() from the all-gather's receive block on the device
        (kueue_tas_host_admit_block): ``block`` a [world, row_words] int32
        tensor (rows [len, quads...]) or a raw device pointer with
        ``row_words``, ``lens`` the rows' lengths.  Same return value."""
        import numpy as np
        if hasattr(block, "data_ptr"):
            ptr, row_words = block.data_ptr(), int(block.shape[1])
        elif hasattr(block, "ctypes"):  # a host array (the CPU emulator's device memory)
            ptr, row_words = block.ctypes.data, int(block.shape[1])
        else:
            ptr = int(block)
        ln = np.ascontiguousarray(lens, dtype=np.int64)
        cap = max(getattr(self, "_n_compiled", 0), 1)  # at most every compiled workload
        while True:
            adm = np.zeros((cap, 2), dtype=np.int32)
            nw = ctypes.c_size_t()
            nd = ctypes.c_size_t()
            rc = self._lib.kueue_tas_host_admit_block(self._h, ptr, row_words, ln.ctypes.data, ln.size,
                                                      adm.ctypes.data, adm.size, ctypes.byref(nw), ctypes.byref(nd))
            if rc == -5 and nw.value > cap:
                cap = nw.value
                continue
            break
        if rc:
            raise RuntimeError(self._err())
        deltas = np.zeros(nd.value, dtype=DELTA_DTYPE)
        if self._lib.kueue_tas_host_last_deltas(self._h, deltas.ctypes.data, deltas.size):
            raise RuntimeError(self._err())
        return adm[: nw.value], deltas

    def last_admit_stats(self):
        """The last admit: (window rounds, candidates walked in order, candidates); -1 for the serial chain."""
        out = (ctypes.c_int64 * 3)()
        if self._lib.kueue_tas_host_last_admit_stats(self._h, out):
            raise RuntimeError(self._err())
        return tuple(out)

    def last_admit_times(self):
        """Host ms of the last admit: (record prep, kueue_tas_admit, delta list)."""
        ms = (ctypes.c_double * 3)()
        self._lib.kueue_tas_host_last_admit_times(self._h, ms)
        return tuple(ms)

    def apply_deltas(self, deltas):
        """Apply another replica's admission deltas (numpy DELTA_DTYPE)."""
        import numpy as np
        d = np.ascontiguousarray(deltas, dtype=DELTA_DTYPE)
        if self._lib.kueue_tas_host_apply_deltas(self._h, d.ctypes.data, d.size):
            raise RuntimeError(self._err())

    def find_topology_assignments_for_workload(self, podsets: list, workload: dict = None,
                                               simulate_empty: bool = False) -> list:
        """FindTopologyAssignmentsForFlavor(..., WithWorkload(wl)) (tas_flavor_snapshot.go:519):
        workload = {"unhealthyNodes": [...], "podSetAssignments": [{"name", "topologyAssignment"}]};
        with unhealthy nodes the PodSets' existing assignments are repaired (node replacement)."""
        doc = dict(workload or {}, podSets=podsets)
        out = ctypes.c_void_p()
        if self._lib.kueue_tas_host_find_workload(self._h, json.dumps(doc).encode(), int(simulate_empty),
                                                  ctypes.byref(out)):
            raise RuntimeError(self._err())
        return _take(self._lib, out)["results"]

    # ---- snapshot queries of the scheduler's other callers ----
    def has_level(self, topology_request) -> bool:
        """TASFlavorSnapshot.HasLevel (tas_flavor_snapshot.go:1065) of a
        PodSetTopologyRequest dict (or None)."""
        r = ctypes.c_int32()
        if self._lib.kueue_tas_host_has_level(self._h, json.dumps(topology_request).encode(), ctypes.byref(r)):
            raise RuntimeError(self._err())
        return bool(r.value)

    def is_topology_assignment_stale(self, assignment: dict):
        """IsTopologyAssignmentStale (:736) of an internal TopologyAssignment:
        (stale, values[0] of the first unknown domain or "")."""
        st = ctypes.c_int32()
        out = ctypes.c_void_p()
        if self._lib.kueue_tas_host_assignment_stale(self._h, json.dumps(assignment).encode(), ctypes.byref(st),
                                                     ctypes.byref(out)):
            raise RuntimeError(self._err())
        d = ctypes.cast(out, ctypes.c_char_p).value.decode()
        self._lib.kueue_tas_free(out)
        return bool(st.value), d

    def serialize_free_capacity_per_domain(self) -> str:
        """SerializeFreeCapacityPerDomain (:320): the JSON text itself."""
        out = ctypes.c_void_p()
        if self._lib.kueue_tas_host_free_capacity_json(self._h, ctypes.byref(out)):
            raise RuntimeError(self._err())
        s = ctypes.cast(out, ctypes.c_char_p).value.decode()
        self._lib.kueue_tas_free(out)
        return s

    def leaf_ids(self) -> list:
        out = ctypes.c_void_p()
        if self._lib.kueue_tas_host_leaf_ids(self._h, ctypes.byref(out)):
            raise RuntimeError(self._err())
        return _take(self._lib, out)

    def select_groups(self):
        """(slot groups of the last chunk's BestFit select, chunks re-run with
        unbounded select lists so far) — kueue_tas_select_groups."""
        g, r = ctypes.c_int64(), ctypes.c_int64()
        self._lib.kueue_tas_select_groups(self.device_ctx(), ctypes.byref(g), ctypes.byref(r))
        return g.value, r.value

    def merge_reruns(self) -> int:
        """Device chunks re-run with the exact phase-1 class merge (kueue_tas_merge_reruns)."""
        self._lib.kueue_tas_merge_reruns.restype = ctypes.c_int64
        self._lib.kueue_tas_merge_reruns.argtypes = [ctypes.c_void_p]
        return int(self._lib.kueue_tas_merge_reruns(self.device_ctx()))

    def device_ctx(self):
        """The kueue_tas_ctx* under this snapshot (for direct device-layer calls)."""
        p = self._lib.kueue_tas_host_ctx(self._h)
        if not p:
            raise RuntimeError(self._err())
        return p

    def compile_workload(self, podsets: list, simulate_empty: bool = False):
        """kueue_tas_host_compile_workload: (reqs buffer, taint table int32 array,
        num_taints, affinity buffer, affinity values int32 array, early reasons)."""
        import numpy as np
        c = ctypes
        ng, tl, na, nv = c.c_size_t(), c.c_size_t(), c.c_size_t(), c.c_size_t()
        nt = c.c_int32()
        doc = json.dumps(podsets).encode()
        rc = self._lib.kueue_tas_host_compile_workload(self._h, doc, int(simulate_empty), None, 0, c.byref(ng), None, 0,
                                                       c.byref(tl), c.byref(nt), None, 0, c.byref(na), None, 0,
                                                       c.byref(nv), None)
        if rc not in (0, -5):
            raise RuntimeError(self._err())
        from . import abi
        reqs = (abi.EvalReq * max(ng.value, 1))()
        taints = np.zeros(max(tl.value, 1), dtype=np.int32)
        aff = (abi.AffinityReq * max(na.value, 1))()
        vals = np.zeros(max(nv.value, 1), dtype=np.int32)
        out = c.c_void_p()
        if self._lib.kueue_tas_host_compile_workload(self._h, doc, int(simulate_empty), reqs, ng.value, c.byref(ng),
                                                     taints.ctypes.data, taints.size, c.byref(tl), c.byref(nt),
                                                     aff, na.value, c.byref(na), vals.ctypes.data,
                                                     vals.size, c.byref(nv), c.byref(out)):
            raise RuntimeError(self._err())
        return reqs, ng.value, taints[: tl.value], nt.value, aff, na.value, vals[: nv.value], _take(self._lib, out)

    RUN_COMPILE = 1  # KUEUE_TAS_RUN_COMPILE: group + compile every TASPodSetRequests in the call
    RUN_VALUES = 2   # KUEUE_TAS_RUN_VALUES: build the TopologyAssignment domains (Values, Count)

    def run_compiled(self, want_hash: bool = False, flags: int = 0):
        """One timed step over the compiled workloads; returns the result hash if asked."""
        h = ctypes.c_uint64()
        rc = self._lib.kueue_tas_host_run(self._h, flags, ctypes.byref(h) if want_hash else None)
        if rc != 0:
            raise RuntimeError(f"kueue_tas_host_run_compiled failed ({rc}): {self._err()}")
        return h.value if want_hash else None
