"""ctypes binding of libdslabs_hip.so (include/dslabs_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).
There is no CPU fallback: if the shared object is missing, importing the search API fails.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# DSL_LIB_VARIANT selects an instrumented in-tree build (e.g. "phases" -> libdslabs_hip_phases.so,
# built by tools/build_variant.sh); the default is the product library.
_VARIANT = os.environ.get("DSL_LIB_VARIANT", "")
LIB_PATH = os.path.join(HERE, "libdslabs_hip%s.so" % ("_" + _VARIANT if _VARIANT else ""))

DSL_MAX_NODES = 32
DSL_MAX_PREDICATES = 16
DSL_MAX_POOL = 48
DSL_MAX_PARAMS = 64
DSL_MAX_EVENT_FIELDS = 8
DSL_PROTO_PINGPONG_IR = 8  # protocols generated from the IR (dslabs_amd/ir/specs)
DSL_PROTO_AMOKV_IR = 9
DSL_PROTO_MULTIPAXOS_IR = 10
DSL_PROTO_PB_IR = 11

# dsl_status
DSL_OK = 0
STATUS_NAMES = {
    -1: "DSL_ERR_ARG", -2: "DSL_ERR_HIP", -3: "DSL_ERR_TABLE_FULL", -4: "DSL_ERR_FRONTIER_FULL",
    -5: "DSL_ERR_STATE_OVERFLOW", -6: "DSL_ERR_UNKNOWN_PROTOCOL", -7: "DSL_ERR_UNKNOWN_PREDICATE",
    -8: "DSL_ERR_COMM", -9: "DSL_ERR_NO_DEVICE",
}

# Exported symbols declared in include/dslabs_hip.h (checked by tests/test_capi.py).
EXPORTED = [
    "dsl_abi_version", "dsl_device_count", "dsl_state_bytes", "dsl_init_state", "dsl_drop_pending_messages",
    "dsl_undrop_messages", "dsl_comm_unique_id", "dsl_create",
    "dsl_set_settings", "dsl_set_initial", "dsl_get_initial", "dsl_run", "dsl_progress",
    "dsl_kernel_stats", "dsl_result_free", "dsl_destroy", "dsl_last_error", "dsl_create_with_host_comm",
    "dsl_run_dfs", "dsl_replay", "dsl_human_readable_trace", "dsl_set_dropped",
]
DSL_ABI_VERSION = 5  # include/dslabs_hip.h; load() refuses a library of another layout


class dsl_protocol_desc(ctypes.Structure):
    _fields_ = [("protocol", ctypes.c_int32), ("n_params", ctypes.c_int32),
                ("params", ctypes.c_int64 * DSL_MAX_PARAMS)]


class dsl_predicate(ctypes.Structure):
    _fields_ = [("pred_id", ctypes.c_int32), ("negate", ctypes.c_int32),
                ("arg0", ctypes.c_int64), ("arg1", ctypes.c_int64)]


class dsl_settings(ctypes.Structure):
    _fields_ = [
        ("max_depth", ctypes.c_int32), ("max_time_ms", ctypes.c_int32),
        ("network_active", ctypes.c_int32), ("deliver_timers", ctypes.c_int32),
        ("link_active", (ctypes.c_int8 * DSL_MAX_NODES) * DSL_MAX_NODES),
        ("sender_active", ctypes.c_int8 * DSL_MAX_NODES),
        ("receiver_active", ctypes.c_int8 * DSL_MAX_NODES),
        ("timers_active", ctypes.c_int8 * DSL_MAX_NODES),
        ("n_invariants", ctypes.c_int32), ("n_goals", ctypes.c_int32), ("n_prunes", ctypes.c_int32),
        ("invariants", dsl_predicate * DSL_MAX_PREDICATES),
        ("goals", dsl_predicate * DSL_MAX_PREDICATES),
        ("prunes", dsl_predicate * DSL_MAX_PREDICATES),
        ("table_log2_slots", ctypes.c_int32), ("n_pool", ctypes.c_int32),
        ("max_frontier_states", ctypes.c_uint64), ("memory_budget_bytes", ctypes.c_uint64),
        ("pool", dsl_predicate * DSL_MAX_POOL),
        ("do_checks", ctypes.c_int32), ("check_sample", ctypes.c_int32),
    ]


DSL_CHECKS_NONE, DSL_CHECKS_ERRORS, DSL_CHECKS_ALL = 0, 1, 2  # dsl_settings.do_checks


class dsl_engine_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("rank", ctypes.c_int32), ("world_size", ctypes.c_int32),
                ("virtual_shards", ctypes.c_int32), ("comm_id", ctypes.c_uint8 * 128),
                ("replicate_below", ctypes.c_int64), ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32)]


DSL_CFG_RCCL_AT_WORLD_1 = 1           # dsl_engine_config.flags
DSL_HOST_COMM_DEVICE_COLLECTIVES = 1  # dsl_host_comm.flags


class dsl_dfs_config(ctypes.Structure):
    _fields_ = [("probes", ctypes.c_int64), ("seed", ctypes.c_uint64), ("max_probes", ctypes.c_int64),
                ("steps_per_launch", ctypes.c_int32), ("max_trace", ctypes.c_int32),
                ("no_minimize", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class dsl_event(ctypes.Structure):
    _fields_ = [("is_timer", ctypes.c_int32), ("from_", ctypes.c_int32), ("to", ctypes.c_int32),
                ("type", ctypes.c_int32), ("n_fields", ctypes.c_int32), ("timer_min", ctypes.c_int32),
                ("timer_max", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("fields", ctypes.c_int64 * DSL_MAX_EVENT_FIELDS)]


class dsl_result(ctypes.Structure):
    _fields_ = [
        ("end_condition", ctypes.c_int32), ("terminal_depth", ctypes.c_int32),
        ("predicate_index", ctypes.c_int32), ("max_depth", ctypes.c_int32),
        ("states", ctypes.c_uint64), ("n_levels", ctypes.c_int32), ("trace_len", ctypes.c_int32),
        ("per_depth", ctypes.POINTER(ctypes.c_uint64)), ("trace", ctypes.POINTER(dsl_event)),
        ("terminal_state", ctypes.POINTER(ctypes.c_uint8)), ("state_bytes", ctypes.c_uint32),
        ("initial_depth", ctypes.c_int32), ("elapsed_s", ctypes.c_double),
        ("successors", ctypes.c_uint64), ("new_states_inserted", ctypes.c_uint64),
        ("exchanged_states", ctypes.c_uint64), ("level_ms_max", ctypes.c_double),
        ("checks_run", ctypes.c_uint64), ("not_deterministic", ctypes.c_uint64), ("not_idempotent", ctypes.c_uint64),
        ("first_not_deterministic", dsl_event), ("first_not_idempotent", dsl_event),
    ]


class dsl_stats(ctypes.Structure):
    _fields_ = [("expand_ms", ctypes.c_double), ("exchange_ms", ctypes.c_double),
                ("expand_launches", ctypes.c_uint64), ("parents", ctypes.c_uint64),
                ("work_items", ctypes.c_uint64), ("new_states", ctypes.c_uint64), ("appended", ctypes.c_uint64),
                ("exchanged", ctypes.c_uint64), ("state_bytes", ctypes.c_uint32), ("world_size", ctypes.c_uint32),
                ("table_slots", ctypes.c_uint64), ("terminal_finds", ctypes.c_uint64),
                ("sharded_levels", ctypes.c_uint64), ("probes", ctypes.c_uint64),
                ("host_syncs", ctypes.c_uint64), ("table_rehashes", ctypes.c_uint64),
                ("rccl_version", ctypes.c_int32), ("level_slots", ctypes.c_int32),
                ("cost_c_ns", ctypes.c_double), ("cost_x_us", ctypes.c_double), ("shard_work_min", ctypes.c_uint64),
                ("exchange_rounds", ctypes.c_uint64), ("fast_levels", ctypes.c_uint64), ("completions", ctypes.c_uint64),
                ("deduped", ctypes.c_uint64)]


_lib = None


def load() -> ctypes.CDLL:
    """Loads the in-tree libdslabs_hip.so; raises loudly when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`. "
            "The MI355X engine has no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    lib.dsl_abi_version.restype = ctypes.c_int
    lib.dsl_device_count.restype = ctypes.c_int
    lib.dsl_state_bytes.argtypes = [P(dsl_protocol_desc)]
    lib.dsl_init_state.argtypes = [P(dsl_protocol_desc), P(ctypes.c_uint8), ctypes.c_size_t]
    lib.dsl_drop_pending_messages.argtypes = [P(dsl_protocol_desc), P(ctypes.c_uint8), ctypes.c_size_t,
                                              P(ctypes.c_uint64), ctypes.c_int32, P(ctypes.c_int32)]
    lib.dsl_undrop_messages.argtypes = [P(dsl_protocol_desc), P(ctypes.c_uint8), ctypes.c_size_t,
                                        P(ctypes.c_uint64), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
    lib.dsl_comm_unique_id.argtypes = [P(ctypes.c_uint8)]
    lib.dsl_create.argtypes = [P(dsl_protocol_desc), P(dsl_engine_config), P(ctypes.c_void_p)]
    lib.dsl_set_settings.argtypes = [ctypes.c_void_p, P(dsl_settings)]
    lib.dsl_set_initial.argtypes = [ctypes.c_void_p, P(ctypes.c_uint8), ctypes.c_size_t, ctypes.c_int32]
    lib.dsl_get_initial.argtypes = [ctypes.c_void_p, P(ctypes.c_uint8), ctypes.c_size_t]
    lib.dsl_set_dropped.argtypes = [ctypes.c_void_p, P(ctypes.c_uint64), ctypes.c_int32]
    lib.dsl_run.argtypes = [ctypes.c_void_p, P(P(dsl_result))]
    lib.dsl_run_dfs.argtypes = [ctypes.c_void_p, P(dsl_dfs_config), P(P(dsl_result))]
    lib.dsl_replay.argtypes = [ctypes.c_void_p, P(dsl_event), ctypes.c_int32, ctypes.c_int32, P(P(dsl_result))]
    lib.dsl_human_readable_trace.argtypes = [ctypes.c_void_p, P(dsl_event), ctypes.c_int32, P(P(dsl_result))]
    lib.dsl_progress.argtypes = [ctypes.c_void_p, P(ctypes.c_uint64), P(ctypes.c_int32)]
    lib.dsl_kernel_stats.argtypes = [ctypes.c_void_p, P(dsl_stats)]
    lib.dsl_create_with_host_comm.argtypes = [P(dsl_protocol_desc), P(dsl_engine_config), ctypes.c_void_p,
                                              P(ctypes.c_void_p)]
    lib.dsl_result_free.argtypes = [P(dsl_result)]
    lib.dsl_result_free.restype = None
    lib.dsl_destroy.argtypes = [ctypes.c_void_p]
    lib.dsl_destroy.restype = None
    lib.dsl_last_error.restype = ctypes.c_char_p
    if lib.dsl_abi_version() != DSL_ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {lib.dsl_abi_version()}, this binding needs {DSL_ABI_VERSION} "
                           "(rebuild the library)")
    _lib = lib
    return lib


class EngineError(RuntimeError):
    def __init__(self, code: int, where: str):
        lib = load()
        msg = lib.dsl_last_error().decode(errors="replace")
        super().__init__(f"{where}: {STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


def check(code: int, where: str) -> None:
    if code != DSL_OK:
        raise EngineError(code, where)
