"""ctypes mirror of the plain-C structs of include/kueue_tas.h (ABI version 5).

For bindings that call the device layer directly (kueue_tas_snapshot_load,
kueue_tas_eval_batch) instead of going through the JSON host layer; the
field order and widths follow the header line by line, and
tests/test_raw_abi.py pins them against the library."""
import ctypes as c

MAX_LEVELS = 16
MAX_COLS = 32
MAX_SELECTORS = 8
MAX_LAYERS = 4

F_REQUIRED = 1
F_UNCONSTRAINED = 2
F_LFC = 4
F_SIMULATE_EMPTY = 8
F_LEADER = 16
F_MULTILAYER = 32
F_AFFINITY = 64
F_DOMAIN = 128
F_SELECTOR_EXT = 256

ST_OK = 0
ST_NO_DOMAINS = 1
ST_NOT_FIT = 2
ST_MULTILAYER = 3
ST_INTERNAL = 4


class SnapshotDesc(c.Structure):  # kueue_tas_snapshot_desc
    _fields_ = [
        ("num_levels", c.c_int32),
        ("level_sizes", c.POINTER(c.c_int32)),
        ("child_offsets", c.POINTER(c.c_int32)),
        ("num_cols", c.c_int32),
        ("free_capacity", c.POINTER(c.c_int64)),
        ("tas_usage", c.POINTER(c.c_int64)),
        ("free_present", c.POINTER(c.c_uint32)),
        ("usage_present", c.POINTER(c.c_uint32)),
        ("lowest_is_hostname", c.c_int32),
        ("taint_profile", c.POINTER(c.c_int32)),
        ("num_label_cols", c.c_int32),
        ("label_values", c.POINTER(c.c_int32)),
        ("domain_id_rank", c.POINTER(c.c_int32)),
    ]


class Delta(c.Structure):  # kueue_tas_delta
    _fields_ = [("leaf", c.c_int32), ("col", c.c_int32), ("delta", c.c_int64)]


class EvalReq(c.Structure):  # kueue_tas_eval_req
    _fields_ = [
        ("flags", c.c_uint32),
        ("count", c.c_int32),
        ("slice_size", c.c_int32),
        ("requested_level", c.c_int32),
        ("slice_level", c.c_int32),
        ("num_req", c.c_int32),
        ("num_leader_req", c.c_int32),
        ("num_selectors", c.c_int32),
        ("req_col", c.c_int32 * MAX_COLS),
        ("req_val", c.c_int64 * MAX_COLS),
        ("leader_col", c.c_int32 * MAX_COLS),
        ("leader_val", c.c_int64 * MAX_COLS),
        ("slice_size_at_level", c.c_int32 * MAX_LEVELS),
        ("sel_col", c.c_int32 * MAX_SELECTORS),
        ("sel_val", c.c_int32 * MAX_SELECTORS),
        ("num_layers", c.c_int32),
        ("layer_level", c.c_int32 * MAX_LAYERS),
        ("layer_size", c.c_int32 * MAX_LAYERS),
        ("taint_table", c.c_int32),
        ("assumed_begin", c.c_int32),
        ("assumed_end", c.c_int32),
        ("affinity_begin", c.c_int32),
        ("affinity_end", c.c_int32),
        ("domain_begin", c.c_int32),
        ("domain_end", c.c_int32),
        ("selector_begin", c.c_int32),
        ("selector_end", c.c_int32),
    ]


class AffinityReq(c.Structure):  # kueue_tas_affinity_req
    _fields_ = [("term", c.c_int32), ("col", c.c_int32), ("negate", c.c_int32), ("begin", c.c_int32),
                ("len", c.c_int32)]


class Assumed(c.Structure):  # kueue_tas_assumed
    _fields_ = [("leaf", c.c_int32), ("col", c.c_int32), ("value", c.c_int64)]


class EvalOut(c.Structure):  # kueue_tas_eval_out
    _fields_ = [
        ("status", c.c_int32),
        ("a", c.c_int32),
        ("b", c.c_int32),
        ("fit_level", c.c_int32),
        ("num_workers", c.c_int32),
        ("num_leaders", c.c_int32),
        ("assignment_nil", c.c_int32),
        ("total_nodes", c.c_int32),
        ("excl_selector", c.c_int32),
        ("excl_affinity", c.c_int32),
        ("excl_topology", c.c_int32),
        ("ml_fit", c.c_int32 * MAX_LAYERS),
        ("ml_need", c.c_int32 * MAX_LAYERS),
        ("reserved", c.c_int32 * 2),
    ]


class Config(c.Structure):  # kueue_tas_config
    _fields_ = [("list_cap", c.c_int32), ("max_batch", c.c_int32), ("device", c.c_int32), ("flags", c.c_int32)]


def bind_device_layer(lib):
    """argtypes of the device-layer entry points the raw bindings call."""
    P = c.POINTER
    lib.kueue_tas_ctx_create.argtypes = [P(Config)]
    lib.kueue_tas_ctx_create.restype = c.c_void_p
    lib.kueue_tas_ctx_destroy.argtypes = [c.c_void_p]
    lib.kueue_tas_ctx_destroy.restype = None
    lib.kueue_tas_last_error.argtypes = [c.c_void_p]
    lib.kueue_tas_last_error.restype = c.c_char_p
    lib.kueue_tas_snapshot_load.argtypes = [c.c_void_p, P(SnapshotDesc)]
    lib.kueue_tas_snapshot_load.restype = c.c_int
    lib.kueue_tas_snapshot_apply_deltas.argtypes = [c.c_void_p, P(Delta), c.c_size_t, c.c_void_p]
    lib.kueue_tas_snapshot_apply_deltas.restype = c.c_int
    lib.kueue_tas_eval_batch.argtypes = [c.c_void_p, P(EvalReq), c.c_size_t, c.c_void_p, c.c_size_t, c.c_int32,
                                         c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t,
                                         P(EvalOut), P(c.c_int64), c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p]
    lib.kueue_tas_eval_batch.restype = c.c_int
    lib.kueue_tas_fetch_entries.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    lib.kueue_tas_fetch_entries.restype = c.c_int
    return lib
