"""ctypes binding of the C ABI in include/pipelinedp_amd.h.

The library is built in-tree (``__graft_entry__.build()``) as
``pipelinedp_amd/lib/libpipelinedp_amd.so``.  There is no CPU fallback: if
the library is missing or fails to load, :func:`lib` raises
:class:`NativeLibraryError`.

torch is imported before the library is loaded so that the library binds to
the same ``libamdhip64.so.7`` instance torch uses (both carry that SONAME);
device pointers and stream handles from torch are then valid here.
"""
import ctypes
import os
import threading

LIB_PATH = os.environ.get("PIPELINEDP_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libpipelinedp_amd.so")

# constants (include/pipelinedp_amd.h)
ABI_VERSION = 14
VALUE_NONE, VALUE_F64, VALUE_I64 = 0, 1, 2
ACC_SUM, ACC_NSUM, ACC_NSUM2, SUM_PER_PARTITION, SUM_INT = 0x1, 0x2, 0x4, 0x8, 0x10
DEBUG_CORRUPT_RECORDS = 0x40000000  # tests only (pipelinedp_amd.h)
PROBE_LEVEL1 = 0x20000000  # placement probe: level 1 only (pipelinedp_amd.h)
SELECT_ALL_NONEMPTY = 0
SELECT_TRUNCATED_GEOMETRIC = 1
SELECT_LAPLACE_THRESHOLDING = 2
SELECT_GAUSSIAN_THRESHOLDING = 3
SELECT_PUBLIC = 4
OP_COUNT, OP_SUM, OP_PRIVACY_ID_COUNT, OP_MEAN, OP_VARIANCE, OP_THRESHOLDED_PID = 1, 2, 3, 4, 5, 6
NOISE_LAPLACE, NOISE_GAUSSIAN = 0, 1
ALGO_AUTO, ALGO_GLOBAL_SKETCH, ALGO_BUCKETED, ALGO_PAIR_TABLE = 0, 1, 2, 3
MERGE_AUTO, MERGE_ATOMIC, MERGE_RANGES = 0, 1, 2
KEYS_AUTO, KEYS_WIDE, KEYS_COMPACT, KEYS_PACKED, KEYS_PACKED_WIDE, KEYS_PACKED64 = 0, 1, 2, 3, 4, 5
MAX_L0 = 2**31 - 1            # pipelinedp_amd.h PDP_MAX_*
MAX_LINF = 2**31 - 1
MAX_CONTRIBUTIONS = 2**31 - 1
MAX_OPS = 8

EXPORTED_SYMBOLS = (
    "pdp_abi_version",
    "pdp_last_error",
    "pdp_bound_workspace_bytes",
    "pdp_bound_plan",
    "pdp_bound_contributions",
    "pdp_reduce_partitions",
    "pdp_select_partitions",
    "pdp_compact_workspace_bytes",
    "pdp_compact",
    "pdp_noise_metrics",
    "pdp_add_noise",
    "pdp_dataset_histograms_workspace_bytes",
    "pdp_dataset_histograms",
    "pdp_dataset_histograms_pairs",
    "pdp_dataset_histograms_exchange_offsets",
    "pdp_dataset_histograms_finish",
    "pdp_dataset_histograms_preaggregated_workspace_bytes",
    "pdp_dataset_histograms_preaggregated",
    "pdp_dataset_histograms_preaggregated_rows",
    "pdp_dataset_histograms_preaggregated_exchange_offsets",
    "pdp_dataset_histograms_preaggregated_finish",
    "pdp_dataset_histograms_preaggregated_weight_offsets",
    "pdp_dataset_histograms_weight_bins",
    "pdp_bound_error_flags",
    "pdp_bound_error_flags_async",
    "pdp_owner_mismatches",
    "pdp_bound_stats_read",
    "pdp_bound_stats_async",
    "pdp_profiler_enable",
    "pdp_profiler_report",
)
PROF_NAME_LEN = 64


class NativeLibraryError(RuntimeError):
    """The HIP library is missing, failed to load, or returned an error."""


class BoundConfig(ctypes.Structure):
    _fields_ = [
        ("n_rows", ctypes.c_int64),
        ("n_privacy_ids", ctypes.c_int64),
        ("n_partitions", ctypes.c_int64),
        ("l0", ctypes.c_int32),
        ("linf", ctypes.c_int32),
        ("value_kind", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("min_value", ctypes.c_double),
        ("max_value", ctypes.c_double),
        ("middle", ctypes.c_double),
        ("min_sum", ctypes.c_double),
        ("max_sum", ctypes.c_double),
        ("row_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("algorithm", ctypes.c_int32),
        ("merge", ctypes.c_int32),
        ("max_contributions", ctypes.c_int32),
        ("rows_are_units", ctypes.c_int32),
        ("key_format", ctypes.c_int32),
        ("sieve", ctypes.c_int32),
        ("sieve_band", ctypes.c_int32),
        ("sieve_threads", ctypes.c_int32),
        ("bucket_threads", ctypes.c_int32),
    ]


class BoundPlanInfo(ctypes.Structure):
    _fields_ = [
        ("algorithm", ctypes.c_int32),
        ("bucket_bits", ctypes.c_int32),
        ("rand_shift", ctypes.c_int32),
        ("pk_bits", ctypes.c_int32),
        ("n_buckets", ctypes.c_int64),
        ("n_tiles", ctypes.c_int64),
        ("lds_bytes", ctypes.c_int64),
        ("merge", ctypes.c_int32),
        ("n_ranges", ctypes.c_int32),
        ("range_group", ctypes.c_int64),
        ("key_format", ctypes.c_int32),
        ("sieve", ctypes.c_int32),
        ("band", ctypes.c_int32),
        ("sieve_threads", ctypes.c_int32),
        ("bucket_threads", ctypes.c_int32),
        ("hist_u16", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class BoundStats(ctypes.Structure):
    _fields_ = [
        ("rows_partitioned", ctypes.c_int64),
        ("unresolved_ids", ctypes.c_int64),
        ("fixup_rows", ctypes.c_int64),
        ("sieve", ctypes.c_int32),
        ("error_flags", ctypes.c_uint32),
        ("band_rows", ctypes.c_int64),
        ("unresolved2_ids", ctypes.c_int64),
        ("fixup2_rows", ctypes.c_int64),
        ("band", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class PartitionAccumulators(ctypes.Structure):
    _fields_ = [
        ("privacy_id_count", ctypes.c_void_p),
        ("count", ctypes.c_void_p),
        ("sum", ctypes.c_void_p),
        ("normalized_sum", ctypes.c_void_p),
        ("normalized_sum_sq", ctypes.c_void_p),
    ]


class NoiseParams(ctypes.Structure):
    """pdp_noise_params: one secure (granularity-snapped) mechanism."""
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("scale", ctypes.c_double),
        ("granularity", ctypes.c_double),
        ("lambda_", ctypes.c_double),
        ("step", ctypes.c_int64),
        ("n", ctypes.c_double),
        ("bound", ctypes.c_double),
        ("coef", ctypes.c_double),
        ("corr", ctypes.c_double),
    ]


class SelectConfig(ctypes.Structure):
    _fields_ = [
        ("n_partitions", ctypes.c_int64),
        ("partition_offset", ctypes.c_int64),
        ("strategy", ctypes.c_int32),
        ("max_rows_per_privacy_id", ctypes.c_int32),
        ("pre_threshold", ctypes.c_int32),
        ("keep_table_len", ctypes.c_int32),
        ("keep_prob", ctypes.c_void_p),
        ("noise", NoiseParams),
        ("threshold", ctypes.c_double),
        ("public_mask", ctypes.c_void_p),
        ("seed", ctypes.c_uint64),
    ]


class MetricOp(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("degenerate", ctypes.c_int32),
        ("out_col", ctypes.c_int32 * 4),
        ("noise", NoiseParams * 3),
        ("middle", ctypes.c_double),
        ("min_value", ctypes.c_double),
        ("sq_min_value", ctypes.c_double),
    ]


HIST_LOG_BINS = 16384
HIST_FORCE_PAIR_TABLE = 0x100  # tests only: value_kind bit (pipelinedp_amd.h)
HIST_FORCE_PAIR_HASH = 0x200   # tests only: skip the privacy-id buckets
HIST_SUM_BUCKETS = 10000
HIST_N_INT = 5
HIST_N_FLOAT = 2


class HistogramBins(ctypes.Structure):
    """pdp_histogram_bins: device output arrays of pdp_dataset_histograms (caller-owned)."""
    _fields_ = [(name, ctypes.c_void_p) for name in (
        "int_count", "int_sum", "int_max", "float_count", "float_sum", "float_max",
        "float_lowers", "float_n_lowers")]


_lock = threading.Lock()
_lib = None


def signatures():
    """{symbol: (restype, argtypes)} of every exported function
    (include/pipelinedp_amd.h); tests/test_integration_doc.py checks
    INTEGRATION.md's ctypes stubs against it."""
    P = ctypes.POINTER
    vp, i64, u64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32
    return {
        "pdp_abi_version": (ctypes.c_int, []),
        "pdp_last_error": (ctypes.c_char_p, []),
        "pdp_bound_workspace_bytes": (ctypes.c_int, [P(BoundConfig), P(u64)]),
        "pdp_bound_contributions": (ctypes.c_int, [P(BoundConfig), vp, vp, vp, vp, vp, u64, vp]),
        "pdp_bound_plan": (ctypes.c_int, [P(BoundConfig), P(BoundPlanInfo)]),
        "pdp_reduce_partitions": (ctypes.c_int, [P(BoundConfig), vp, vp, u64, P(PartitionAccumulators), vp]),
        "pdp_select_partitions": (ctypes.c_int, [P(SelectConfig), vp, vp, vp, vp]),
        "pdp_compact_workspace_bytes": (ctypes.c_int, [i64, P(u64)]),
        "pdp_compact": (ctypes.c_int, [vp, i64, vp, vp, vp, u64, vp]),
        "pdp_noise_metrics": (ctypes.c_int, [P(MetricOp), i32, vp, i64, vp, i64,
                                             P(PartitionAccumulators), i32, vp, vp, i64, u64, vp]),
        "pdp_add_noise": (ctypes.c_int, [vp, i32, i64, P(NoiseParams), u64, i64, vp, vp]),
        "pdp_dataset_histograms_workspace_bytes": (ctypes.c_int, [i64, i64, i64, P(u64)]),
        "pdp_dataset_histograms": (ctypes.c_int, [vp, vp, vp, i32, i64, i64, i64, P(HistogramBins),
                                                  vp, u64, vp]),
        "pdp_dataset_histograms_pairs": (ctypes.c_int, [vp, vp, vp, i32, i64, i64, i64, P(HistogramBins),
                                                        vp, u64, vp]),
        "pdp_dataset_histograms_exchange_offsets": (ctypes.c_int, [i64, i64, i64, P(u64), P(u64), P(u64)]),
        "pdp_dataset_histograms_finish": (ctypes.c_int, [i32, i64, i64, i64, i32, P(HistogramBins),
                                                         vp, u64, vp]),
        "pdp_dataset_histograms_preaggregated_workspace_bytes": (ctypes.c_int, [i64, i64, P(u64)]),
        "pdp_dataset_histograms_preaggregated": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, P(HistogramBins),
                                                                vp, u64, vp]),
        "pdp_dataset_histograms_preaggregated_rows": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64,
                                                                     P(HistogramBins), vp, u64, vp]),
        "pdp_dataset_histograms_preaggregated_exchange_offsets": (ctypes.c_int, [i64, i64, P(u64), P(u64),
                                                                                 P(u64), P(u64)]),
        "pdp_dataset_histograms_preaggregated_finish": (ctypes.c_int, [vp, i64, i64, i32, P(HistogramBins),
                                                                       vp, u64, vp]),
        "pdp_dataset_histograms_preaggregated_weight_offsets": (ctypes.c_int, [i64, i64, P(u64), P(u64), P(u64)]),
        "pdp_dataset_histograms_weight_bins": (ctypes.c_int, [vp, vp, i64, P(HistogramBins), vp]),
        "pdp_bound_error_flags": (ctypes.c_int, [vp, P(ctypes.c_uint32), vp]),
        "pdp_bound_error_flags_async": (ctypes.c_int, [vp, vp, vp]),
        "pdp_owner_mismatches": (ctypes.c_int, [vp, i64, i32, i32, vp, vp]),
        "pdp_bound_stats_read": (ctypes.c_int, [P(BoundConfig), vp, u64, P(BoundStats), vp]),
        "pdp_bound_stats_async": (ctypes.c_int, [P(BoundConfig), vp, u64, vp, vp]),
        "pdp_profiler_enable": (ctypes.c_int, [ctypes.c_int]),
        "pdp_profiler_report": (ctypes.c_int, [i32, ctypes.c_char_p, P(ctypes.c_double), P(i64), P(i32)]),
    }


def _declare(lib):
    for name, (res, args) in signatures().items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Loads (once) and returns the native library; raises NativeLibraryError."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"HIP library not built: {LIB_PATH} is missing. Run "
                "`python -c 'import __graft_entry__ as g; g.build()'` first. "
                "pipelinedp_amd has no CPU fallback.")
        import torch  # noqa: F401  (bind to torch's libamdhip64.so.7 first)
        try:
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        missing = [s for s in EXPORTED_SYMBOLS if not hasattr(handle, s)]
        if missing:
            raise NativeLibraryError(f"{LIB_PATH} lacks symbols {missing}")
        _declare(handle)
        if handle.pdp_abi_version() != ABI_VERSION:
            raise NativeLibraryError("ABI version mismatch; rebuild the library")
        _lib = handle
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().pdp_last_error()
        msg = msg.decode() if msg else ""
        raise NativeLibraryError(f"{what} failed with code {rc}: {msg}")


def profiler_enable(on: bool = True):
    """Starts (clears) or stops per-kernel HIP-event timing in the library."""
    check(lib().pdp_profiler_enable(1 if on else 0), "pdp_profiler_enable")


def profiler_report(max_entries: int = 64):
    """{kernel name: (total ms, launches)} since profiler_enable (synchronises)."""
    names = ctypes.create_string_buffer(max_entries * PROF_NAME_LEN)
    total = (ctypes.c_double * max_entries)()
    calls = (ctypes.c_int64 * max_entries)()
    n = ctypes.c_int32(0)
    check(lib().pdp_profiler_report(max_entries, names, total, calls, ctypes.byref(n)),
          "pdp_profiler_report")
    out = {}
    for k in range(n.value):
        raw = names.raw[k * PROF_NAME_LEN:(k + 1) * PROF_NAME_LEN]
        out[raw.split(b"\0", 1)[0].decode()] = (total[k], calls[k])
    return out
