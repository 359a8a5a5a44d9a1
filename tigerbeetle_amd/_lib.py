"""Loader for the in-tree HIP engine library (libtbgpu.so) and its C ABI (include/tbgpu.h).

The library is built in-tree by `tigerbeetle_amd.build` (hipcc --offload-arch=gfx950).  There is
no CPU fallback: if the library is missing or no GPU is visible, calls fail loudly.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libtbgpu.so")
# A/B timing experiments (tools/gpu/ab.sh) load an older build of the same library.
AB_PATH = os.environ.get("TBGPU_AB_LIB")

STATUS_OK, STATUS_INVALID, STATUS_PANIC, STATUS_DEVICE = 0, 1, 2, 3

CONFIG_PROFILE = 1
CONFIG_SEQUENTIAL_FALLBACK = 2
CONFIG_SWEEP_EARLY = 4
CONFIG_SWEEP_OFF = 8
CONFIG_SWEEP_WINDOW = 16


class tbgpu_config(ctypes.Structure):
    _fields_ = [
        ("accounts_max", ctypes.c_uint64),
        ("transfers_max", ctypes.c_uint64),
        ("pass_events_max", ctypes.c_uint32),
        ("pass_batches_max", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("device_count", ctypes.c_uint32),
        ("devices", ctypes.c_int32 * 16),  # TBGPU_DEVICES_MAX
    ]


class tbgpu_delta_counts(ctypes.Structure):
    _fields_ = [("accounts", ctypes.c_uint64), ("transfers", ctypes.c_uint64), ("posted", ctypes.c_uint64),
                ("created_after", ctypes.c_uint64)]


class tbgpu_stats(ctypes.Structure):
    _fields_ = [
        ("passes", ctypes.c_uint64),
        ("events", ctypes.c_uint64),
        ("dependent_events", ctypes.c_uint64),
        ("accounts", ctypes.c_uint64),
        ("transfers", ctypes.c_uint64),
        ("ms_validate", ctypes.c_double),
        ("ms_resolve", ctypes.c_double),
        ("ms_replay", ctypes.c_double),
        ("ms_clear", ctypes.c_double),
        ("launches_validate", ctypes.c_uint64),
        ("launches_resolve", ctypes.c_uint64),
        ("launches_replay", ctypes.c_uint64),
        ("launches_clear", ctypes.c_uint64),
        ("ms_apply", ctypes.c_double),
        ("launches_apply", ctypes.c_uint64),
        ("flow_passes", ctypes.c_uint64),
        ("flow_units", ctypes.c_uint64),
        ("flow_runs", ctypes.c_uint64),
        ("flow_run_units", ctypes.c_uint64),
        ("flow_plan_ms", ctypes.c_double),
        ("flow_run_ms", ctypes.c_double),
        ("bounds_passes", ctypes.c_uint64),
        ("bounds_units", ctypes.c_uint64),
        ("bounds_rounds", ctypes.c_uint64),
        ("bounds_skipped", ctypes.c_uint64),
        ("bounds_abandoned", ctypes.c_uint64),
        ("bounds_swept", ctypes.c_uint64),
        ("sweep_ms", ctypes.c_double),
        ("sweep_loop_ms", ctypes.c_double),
        ("sweep_wait_ms", ctypes.c_double),
        ("sweep_u64_passes", ctypes.c_uint64),
        ("flow_exec_ms", ctypes.c_double),
        ("flow_phase_ms", ctypes.c_double * 8),
        ("walk_segments", ctypes.c_uint64),
        ("walk_heavy", ctypes.c_uint64),
        ("walk_heavy_positions", ctypes.c_uint64),
        ("walk_heavy_windows", ctypes.c_uint64),
        ("walk_heavy_stops", ctypes.c_uint64),
        ("walk_heavy_blocks", ctypes.c_uint64),
        ("walk_heavy_blocked_ms", ctypes.c_double),
        ("walk_longest", ctypes.c_uint64),
        ("walk_crit_windows", ctypes.c_uint64),
        ("walk_crit_blocks", ctypes.c_uint64),
        ("walk_crit_wait_ms", ctypes.c_double),
        ("walk_crit_ms", ctypes.c_double),
        ("walk_dbg", ctypes.c_uint64 * 4),
        ("span_ms", ctypes.c_double * 3),
        ("span_launches", ctypes.c_uint64 * 3),
        ("node_passes_clean", ctypes.c_uint64),
        ("node_passes_split", ctypes.c_uint64),
        ("node_passes_whole", ctypes.c_uint64),
        ("node_sequenced_events", ctypes.c_uint64),
        ("account_table_bytes", ctypes.c_uint64),
        ("node_shard_account_bytes", ctypes.c_uint64 * 16),
        ("transfers_evicted", ctypes.c_uint64),
        ("log_used", ctypes.c_uint64),
        ("log_capacity", ctypes.c_uint64),
        ("write_backs_async", ctypes.c_uint64),
        ("write_backs_bound", ctypes.c_uint64),
    ]


class tbgpu_workload(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("account_count", ctypes.c_uint64),
        ("kind", ctypes.c_uint32),
        ("limit_permille", ctypes.c_uint32),
        ("zipf_s", ctypes.c_double),
        ("hot_limited", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


class tbgpu_ledger_summary(ctypes.Structure):
    _fields_ = [("sums", ctypes.c_uint64 * 8), ("accounts", ctypes.c_uint64), ("stray", ctypes.c_uint64)]


WORLD_MAX = 64
DIRTY_FLAGS, DIRTY_LIMIT = 1, 2
CERT_U128, CERT_U64 = 1, 2


class tbgpu_route_plan(ctypes.Structure):
    _fields_ = [
        ("send_counts", ctypes.c_uint64 * WORLD_MAX),
        ("sum_lo", ctypes.c_uint64),
        ("sum_hi", ctypes.c_uint64),
        ("bound_lo", ctypes.c_uint64),
        ("bound_hi", ctypes.c_uint64),
        ("dirty", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


# Every symbol declared in include/*.h: (name, restype, argtypes).
_P = ctypes.c_void_p
_U8, _U32, _U64 = ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64
SIGNATURES = [
    ("tbgpu_init", ctypes.c_int, [ctypes.POINTER(tbgpu_config), ctypes.POINTER(_P)]),
    ("tbgpu_deinit", None, [_P]),
    ("tbgpu_reset", ctypes.c_int, [_P]),
    ("tbgpu_commit", ctypes.c_int, [_P, _U8, _U64, _P, _U32, _P, _U32, ctypes.POINTER(_U32)]),
    ("tbgpu_prefetch", ctypes.c_int, [_P, _U8, _P, _U32]),
    ("tbgpu_commit_many", ctypes.c_int, [_P, _U8, _U32, ctypes.POINTER(_U64), ctypes.POINTER(_P),
                                         ctypes.POINTER(_U32), ctypes.POINTER(_P), ctypes.POINTER(_U32)]),
    ("tbgpu_commit_pipelined", ctypes.c_int, [_P, _U8, _U32, ctypes.POINTER(_U64), ctypes.POINTER(_P),
                                              ctypes.POINTER(_U32), ctypes.POINTER(_P), ctypes.POINTER(_U32), _U32, _P]),
    ("tbgpu_commit_device_async", ctypes.c_int, [_P, _U8, _U32, ctypes.POINTER(_U64), ctypes.POINTER(_U32),
                                                 _P, _P, _P]),
    ("tbgpu_sync", ctypes.c_int, [_P]),
    ("tbgpu_commit_timestamp", _U64, [_P]),
    ("tbgpu_test_set_balances", ctypes.c_int, [_P, _U64, _U64, ctypes.POINTER(_U64)]),
    ("tbgpu_export_accounts", ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    ("tbgpu_export_transfers", ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    ("tbgpu_export_posted", ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    ("tbgpu_get_stats", ctypes.c_int, [_P, ctypes.POINTER(tbgpu_stats)]),
    ("tbgpu_reset_stats", None, [_P]),
    ("tbgpu_last_error", ctypes.c_char_p, []),
    ("tbgpu_checksum", None, [_P, _U64, _P]),
    ("tbgpu_debug_allocations", _U64, []),
    ("tbgpu_bench_generate_accounts", ctypes.c_int, [_P, _P, _U64, _U64, ctypes.POINTER(tbgpu_workload)]),
    ("tbgpu_bench_generate_transfers", ctypes.c_int, [_P, _P, _U64, _U64, ctypes.POINTER(tbgpu_workload)]),
    ("tbgpu_bench_reset_transfers", ctypes.c_int, [_P]),
    ("tbgpu_bench_pass_latencies", ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    ("tbgpu_bench_profile_mask", ctypes.c_int, [_P, _U32]),
    ("tbgpu_bench_legs_min_events", ctypes.c_int, [_P, _U32]),
    ("tbgpu_bench_walk_merge_max", ctypes.c_int, [_P, _U32]),
    ("tbgpu_bench_flow_launch", ctypes.c_int, [_P, _U32]),
    ("tbgpu_bench_access_mix", ctypes.c_int, [_P, _U64, ctypes.POINTER(ctypes.c_double)]),
    ("tbgpu_bench_ledger_summary", ctypes.c_int, [_P, ctypes.POINTER(tbgpu_ledger_summary)]),
    ("tbgpu_bench_checkpoint_mark", ctypes.c_int, [_P]),
    ("tbgpu_bench_node_shard", ctypes.c_int, [_P, _U32, ctypes.POINTER(_P)]),
    ("tbgpu_device_alloc", ctypes.c_int, [_P, _U64, ctypes.POINTER(_P)]),
    ("tbgpu_device_free", ctypes.c_int, [_P, _P]),
    ("tbgpu_copy_to_host", ctypes.c_int, [_P, _P, _P, _U64]),
    ("tbgpu_register_host", ctypes.c_int, [_P, _P, _U64]),
    ("tbgpu_checkpoint_delta", ctypes.c_int, [_P, _P, _P, _U64, _P, _U64, _P, _U64, _P]),
    ("tbgpu_checkpoint_delta_async", ctypes.c_int, [_P, _P, _P, _U64, _P, _U64, _P, _U64]),
    ("tbgpu_checkpoint_delta_wait", ctypes.c_int, [_P, _P]),
    ("tbgpu_load_accounts", ctypes.c_int, [_P, _P, _U32]),
    ("tbgpu_load_transfers", ctypes.c_int, [_P, _P, _P, _U32]),
    ("tbgpu_set_commit_timestamp", ctypes.c_int, [_P, _U64]),
    ("tbgpu_evict_transfers", ctypes.c_int, [_P, _U64, ctypes.POINTER(_U64)]),
    ("tbgpu_log_window", ctypes.c_int, [_P, _U64, ctypes.POINTER(ctypes.c_void_p)]),
    ("tbgpu_transfers_maybe_cold", ctypes.c_int, [_P, _P, _U32, _P]),
    ("tbgpu_unregister_host", ctypes.c_int, [_P, _P]),
    ("tbgpu_copy_to_device", ctypes.c_int, [_P, _P, _P, _U64]),
    ("tbgpu_marker", ctypes.c_int, [_P, _U32]),
    ("tbgpu_marker_elapsed_ms", ctypes.c_double, [_P, _U32, _U32]),
    # include/tbgpu_shard.h
    ("tbgpu_home", _U32, [_U64, _U64, _U32]),
    ("tbgpu_homes", None, [_P, _U64, _U32, _P]),
    ("tbgpu_route_init", ctypes.c_int, [_P, _U32, _U64]),
    ("tbgpu_route_plan_build", ctypes.c_int, [_P, _U32, ctypes.POINTER(_U64), ctypes.POINTER(_U32), _P, _P, _P, _P,
                                              ctypes.POINTER(tbgpu_route_plan)]),
    ("tbgpu_route_homes", ctypes.c_int, [_P, _P, _U64, _U32, _P]),
    ("tbgpu_route_dependents", ctypes.c_int, [_P, _U32, ctypes.POINTER(_U32), _P, _P, _U32, _P]),
    ("tbgpu_commit_routed_async", ctypes.c_int, [_P, _U64, _P, _U64, _U32, _P]),
    ("tbgpu_commit_routed_owner_async", ctypes.c_int, [_P, _U64, _P, _U64, _U32, _P, _U32, _U32, _P, _U64, _P]),
    ("tbgpu_apply_owner_legs_async", ctypes.c_int, [_P, _P, _U64, _U32]),
    ("tbgpu_route_replies_async", ctypes.c_int, [_P, _U32, ctypes.POINTER(_U32), _P, _P, _P, _P]),
    ("tbgpu_fetch_accounts", ctypes.c_int, [_P, _P, _U32, _P, _P]),
    ("tbgpu_fetch_transfers", ctypes.c_int, [_P, _P, _U32, _P, _P]),
    ("tbgpu_upsert_accounts", ctypes.c_int, [_P, _P, _U32]),
    ("tbgpu_upsert_transfers", ctypes.c_int, [_P, _P, _P, _U32]),
]

_lib = None


class EngineError(RuntimeError):
    def __init__(self, status, message):
        super().__init__("tbgpu status %d: %s" % (status, message))
        self.status = status


class EnginePanic(EngineError):
    """The reference would have panicked (assert / ReleaseSafe overflow trap)."""


def load():
    """Load libtbgpu.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("tigerbeetle_amd: %s is missing — run `python -c 'import __graft_entry__ as g; "
                              "g.build()'` (hipcc --offload-arch=gfx950)" % LIB_PATH)
        lib = ctypes.CDLL(AB_PATH or LIB_PATH)
        for name, res, args in SIGNATURES:
            if AB_PATH and not hasattr(lib, name):
                continue  # an older build: symbols added since are absent
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(status):
    if status == STATUS_OK:
        return
    msg = load().tbgpu_last_error().decode(errors="replace")
    if status == STATUS_PANIC:
        raise EnginePanic(status, msg)
    raise EngineError(status, msg)


def checksum(data):
    """vsr.checksum (src/vsr/checksum.zig:50) of bytes -> int (u128), computed by the library."""
    data = bytes(data)
    out = ctypes.create_string_buffer(16)
    load().tbgpu_checksum(data, len(data), out)
    return int.from_bytes(out.raw, "little")
