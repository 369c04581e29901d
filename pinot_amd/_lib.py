"""ctypes binding of libpinot_hip.so (include/pinot_hip.h).

This is the Python twin of the Java FFM binding shown in INTEGRATION.md. The product path has
no CPU fallback: if the library cannot be loaded, or no GPU is present, calls raise.
"""
import ctypes
import struct
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PHIP_LIB") or os.path.join(_HERE, "libpinot_hip.so")  # PHIP_LIB: A/B builds

PHIP_OK = 0
PHIP_ERR_INVALID = 1
PHIP_ERR_HIP = 2
PHIP_ERR_UNSUPPORTED = 3
PHIP_ERR_NOT_FOUND = 4
PHIP_ERR_NO_DEVICE = 5
PHIP_ERR_TIMEOUT = 6
PHIP_ERR_CANCELLED = 7

FWD_FIXED_BIT, FWD_SORTED, FWD_RAW_CHUNK, FWD_HLL_REGISTERS = 0, 1, 2, 3
NODE_LEAF, NODE_AND, NODE_OR, NODE_NOT = 0, 1, 2, 3
LEAF_MATCH_ALL, LEAF_MATCH_NONE, LEAF_DICT_RANGE, LEAF_DICT_SET, LEAF_DOC_RANGES, LEAF_INVERTED, LEAF_RAW_RANGE, \
    LEAF_RAW_SET, LEAF_RAW_STRING_RANGE, LEAF_RAW_STRING_SET, LEAF_NULL = range(11)


class RawRange(ctypes.Structure):
    """phip_raw_range (include/pinot_hip.h)."""
    _fields_ = [("lo_int", ctypes.c_int64), ("hi_int", ctypes.c_int64), ("lo_real", ctypes.c_double),
                ("hi_real", ctypes.c_double), ("lo_inclusive", ctypes.c_int32), ("hi_inclusive", ctypes.c_int32)]


AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_HLL = range(5)
EXPR_COLUMN, EXPR_ADD, EXPR_SUB, EXPR_MUL = range(4)

EXPORTED_SYMBOLS = (
    "phip_init", "phip_shutdown", "phip_device_count", "phip_last_error", "phip_version",
    "phip_segment_load", "phip_segment_unload", "phip_segment_device_bytes", "phip_query",
    "phip_result_dictionary", "phip_result_free", "phip_filter_bitmap", "phip_plan_create", "phip_plan_execute",
    "phip_plan_destroy", "phip_global_dictionary", "phip_plan_execute_partial", "phip_plan_finish",
    "phip_runtime_versions", "phip_plan_abandon_partial", "phip_result_select_dictionary",
    "phip_plan_set_deadline", "phip_plan_cancel", "phip_plan_exchange",
)

# phip_plan_exchange kinds (include/pinot_hip.h "node plans")
EXCHANGE_NONE = 0
EXCHANGE_RCCL = 1
EXCHANGE_PEER = 2
EXCHANGE_RECORDS = 3
EXCHANGE_HASH = 4

u8p = ctypes.POINTER(ctypes.c_uint8)


class ColumnDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data_type", ctypes.c_int32), ("fwd_kind", ctypes.c_int32),
                ("cardinality", ctypes.c_int32), ("bits_per_value", ctypes.c_int32),
                ("string_width", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("forward", ctypes.c_void_p), ("forward_bytes", ctypes.c_uint64),
                ("dictionary", ctypes.c_void_p), ("dictionary_bytes", ctypes.c_uint64),
                ("inverted", ctypes.c_void_p), ("inverted_bytes", ctypes.c_uint64),
                ("null_vector", ctypes.c_void_p), ("null_vector_bytes", ctypes.c_uint64)]


class SegmentDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("device", ctypes.c_int32), ("num_docs", ctypes.c_int32),
                ("num_columns", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("columns", ctypes.POINTER(ColumnDesc))]


class FilterNode(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("num_children", ctypes.c_int32), ("leaf_kind", ctypes.c_int32),
                ("column", ctypes.c_int32), ("lo", ctypes.c_int32), ("hi", ctypes.c_int32),
                ("exclusive", ctypes.c_int32), ("count", ctypes.c_int32),
                ("ids", ctypes.POINTER(ctypes.c_int32))]


class Aggregation(ctypes.Structure):
    _fields_ = [("function", ctypes.c_int32), ("expr", ctypes.c_int32), ("column_a", ctypes.c_int32),
                ("column_b", ctypes.c_int32), ("log2m", ctypes.c_int32), ("program", ctypes.c_int32)]


class OrderTerm(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("a", ctypes.c_int32), ("b", ctypes.c_int32), ("desc", ctypes.c_int32)]


ORDER_GROUP_KEY, ORDER_VALUE, ORDER_AVG, ORDER_RANGE, ORDER_HLL = 0, 1, 2, 3, 4


class SelectExpr(ctypes.Structure):
    _fields_ = [("expr", ctypes.c_int32), ("column_a", ctypes.c_int32), ("column_b", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class QueryDesc(ctypes.Structure):
    _fields_ = [("num_columns", ctypes.c_int32), ("num_segments", ctypes.c_int32),
                ("columns", ctypes.POINTER(ctypes.c_char_p)), ("segments", ctypes.POINTER(ctypes.c_uint64)),
                ("filter_offsets", ctypes.POINTER(ctypes.c_int32)), ("filter_nodes", ctypes.POINTER(FilterNode)),
                ("num_aggregations", ctypes.c_int32), ("num_group_by", ctypes.c_int32),
                ("aggregations", ctypes.POINTER(Aggregation)), ("group_by_columns", ctypes.POINTER(ctypes.c_int32)),
                ("num_groups_limit", ctypes.c_int64),
                ("order_by_aggregation", ctypes.c_int32), ("order_by_desc", ctypes.c_int32),
                ("trim_size", ctypes.c_int64), ("num_order_by_keys", ctypes.c_int32), ("null_group_by", ctypes.c_int32),
                ("order_by_keys", ctypes.POINTER(ctypes.c_int32)),
                ("num_order_terms", ctypes.c_int32), ("num_filter_programs", ctypes.c_int32),
                ("order_terms", ctypes.POINTER(OrderTerm)),
                ("num_select", ctypes.c_int32), ("stats_programs", ctypes.c_uint32),
                ("select", ctypes.POINTER(SelectExpr)), ("select_limit", ctypes.c_int64)]


class Result(ctypes.Structure):
    _fields_ = [("num_docs_scanned", ctypes.c_int64), ("num_entries_scanned_in_filter", ctypes.c_int64),
                ("num_entries_scanned_post_filter", ctypes.c_int64), ("num_total_docs", ctypes.c_int64),
                ("num_segments_processed", ctypes.c_int32), ("num_segments_matched", ctypes.c_int32),
                ("num_groups_limit_reached", ctypes.c_int32), ("num_aggregations", ctypes.c_int32),
                ("num_groups", ctypes.c_int64), ("num_group_by", ctypes.c_int32), ("num_hll", ctypes.c_int32),
                ("values", ctypes.POINTER(ctypes.c_double)), ("long_values", ctypes.POINTER(ctypes.c_int64)),
                ("hll_registers", ctypes.POINTER(ctypes.c_uint8)), ("group_keys", ctypes.POINTER(ctypes.c_int32)),
                ("scan_kernel_ms", ctypes.c_double), ("device_ms", ctypes.c_double),
                ("num_groups_trimmed", ctypes.c_int32), ("fused", ctypes.c_int32),
                ("long_exact", ctypes.POINTER(ctypes.c_int32)),
                ("filter_kernel_ms", ctypes.c_double), ("agg_kernel_ms", ctypes.c_double),
                ("filter_bytes", ctypes.c_int64), ("agg_bytes", ctypes.c_int64),
                ("num_rows", ctypes.c_int64), ("num_select", ctypes.c_int32), ("reserved_select", ctypes.c_int32),
                ("select_types", ctypes.POINTER(ctypes.c_int32)), ("select_values", ctypes.POINTER(ctypes.c_uint64)),
                ("segment_docs_matched", ctypes.POINTER(ctypes.c_int64)), ("stream_bytes", ctypes.c_int64),
                ("program_docs_matched", ctypes.POINTER(ctypes.c_int64))]


# phip_result's scalar image in one read (the aggregation-only fast path of plan._block_from_result): the fields in
# declaration order, natural alignment (checked against ctypes below)
RESULT_IMAGE = struct.Struct("<4q4iq2i4Q2d2iQ2d3q2i3QqQ")
assert RESULT_IMAGE.size == ctypes.sizeof(Result)


class DictionaryView(ctypes.Structure):
    _fields_ = [("data_type", ctypes.c_int32), ("cardinality", ctypes.c_int32), ("string_width", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("values", ctypes.c_void_p)]


ROW_COUNT, ROW_SUM_I64, ROW_SUM_F64, ROW_MIN, ROW_MAX, ROW_HLL = range(6)
PARTIAL_MAX_ROWS = 9


class Partial(ctypes.Structure):
    """phip_partial: a GPU's dense partial group table (device pointers), merged by the caller."""
    _fields_ = [("num_groups", ctypes.c_int64), ("num_rows", ctypes.c_int32), ("num_hll", ctypes.c_int32),
                ("log2m", ctypes.c_int32), ("device", ctypes.c_int32),
                ("table", ctypes.c_void_p), ("hll", ctypes.c_void_p),
                ("row_kinds", ctypes.c_int32 * PARTIAL_MAX_ROWS), ("global_keys", ctypes.c_int32),
                ("stats", ctypes.c_int64 * 6), ("stats_dev", ctypes.c_void_p), ("hll_u8", ctypes.c_int32),
                ("reserved_partial", ctypes.c_int32)]


class PhipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pinot_hip error {code}: {msg}")
        self.code = code


class UnsupportedOnGpu(Exception):
    """Query shape outside the GPU subset (the Java side would call super.makeInstancePlan)."""


class PhipUnsupported(PhipError, UnsupportedOnGpu):
    """PHIP_ERR_UNSUPPORTED from the library: the plan maker's CPU operator answers the query."""


class QueryTimeoutError(PhipError):
    """PHIP_ERR_TIMEOUT: the plan's deadline passed (QueryTimeoutException / QueryErrorCode.EXECUTION_TIMEOUT,
    BaseSingleBlockCombineOperator.java:137-144)."""


class QueryCancelledError(PhipError):
    """PHIP_ERR_CANCELLED: phip_plan_cancel stopped the execution (QueryCancelledException)."""


_ERRORS = {PHIP_ERR_UNSUPPORTED: PhipUnsupported, PHIP_ERR_TIMEOUT: QueryTimeoutError,
           PHIP_ERR_CANCELLED: QueryCancelledError}


_lib = None
_torch_first = False  # torch's HIP runtime was in the process before the library bound to one


def load(with_torch: bool = False):
    """Load libpinot_hip.so (fails loudly: there is no CPU fallback on the product path).

    One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (same soname), so a process that also
    uses torch on the GPU (RCCL merges, engine/distributed.py) must import torch BEFORE the library loads; the
    library then binds to torch's runtime. ``with_torch`` (or PINOT_AMD_WITH_TORCH=1) does that import; a process
    that already imported torch gets it implicitly. Plain users of the library skip torch's import and keep the
    ROCm runtime the library was built against. Either way the runtime's major version must equal the build's
    (phip_version reports both), else the load fails.
    """
    global _lib, _torch_first
    import sys
    want_torch = with_torch or os.environ.get("PINOT_AMD_WITH_TORCH") == "1"
    if _lib is not None:
        if want_torch and not _torch_first:
            raise RuntimeError("libpinot_hip.so was loaded before torch: its HIP runtime is not torch's. Import torch "
                               "(or call pinot_amd._lib.load(with_torch=True)) before the first load")
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    if want_torch:
        import torch  # noqa: F401
    _torch_first = "torch" in sys.modules
    lib = ctypes.CDLL(LIB_PATH)
    i32, u64, i64 = ctypes.c_int32, ctypes.c_uint64, ctypes.c_int64
    lib.phip_init.argtypes = [ctypes.POINTER(i32), i32]
    lib.phip_init.restype = i32
    lib.phip_shutdown.argtypes = []
    lib.phip_shutdown.restype = i32
    lib.phip_device_count.argtypes = [ctypes.POINTER(i32)]
    lib.phip_device_count.restype = i32
    lib.phip_last_error.argtypes = []
    lib.phip_last_error.restype = ctypes.c_char_p
    lib.phip_version.argtypes = []
    lib.phip_version.restype = ctypes.c_char_p
    lib.phip_segment_load.argtypes = [ctypes.POINTER(SegmentDesc), ctypes.POINTER(u64)]
    lib.phip_segment_load.restype = i32
    lib.phip_segment_unload.argtypes = [u64]
    lib.phip_segment_unload.restype = i32
    lib.phip_segment_device_bytes.argtypes = [u64, ctypes.POINTER(u64)]
    lib.phip_segment_device_bytes.restype = i32
    lib.phip_query.argtypes = [ctypes.POINTER(QueryDesc), ctypes.POINTER(ctypes.POINTER(Result))]
    lib.phip_query.restype = i32
    lib.phip_result_dictionary.argtypes = [ctypes.POINTER(Result), i32, ctypes.POINTER(DictionaryView)]
    lib.phip_result_dictionary.restype = i32
    lib.phip_result_select_dictionary.argtypes = [ctypes.POINTER(Result), i32, ctypes.POINTER(DictionaryView)]
    lib.phip_result_select_dictionary.restype = i32
    lib.phip_result_free.argtypes = [ctypes.POINTER(Result)]
    lib.phip_result_free.restype = None
    lib.phip_filter_bitmap.argtypes = [ctypes.POINTER(QueryDesc), ctypes.POINTER(u64), i64]
    lib.phip_filter_bitmap.restype = i32
    lib.phip_plan_create.argtypes = [ctypes.POINTER(QueryDesc), ctypes.POINTER(u64)]
    lib.phip_plan_create.restype = i32
    lib.phip_plan_execute.argtypes = [u64, ctypes.POINTER(ctypes.POINTER(Result))]
    lib.phip_plan_execute.restype = i32
    lib.phip_plan_destroy.argtypes = [u64]
    lib.phip_plan_destroy.restype = i32
    lib.phip_plan_exchange.argtypes = [u64, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    lib.phip_plan_exchange.restype = i32
    lib.phip_global_dictionary.argtypes = [i32, ctypes.c_char_p, i32, i32, i32, ctypes.c_void_p]
    lib.phip_global_dictionary.restype = i32
    lib.phip_plan_execute_partial.argtypes = [u64, ctypes.POINTER(Partial)]
    lib.phip_plan_execute_partial.restype = i32
    lib.phip_plan_finish.argtypes = [u64, ctypes.POINTER(Partial), ctypes.POINTER(ctypes.POINTER(Result))]
    lib.phip_plan_finish.restype = i32
    lib.phip_plan_abandon_partial.argtypes = [u64]
    lib.phip_plan_abandon_partial.restype = i32
    lib.phip_plan_set_deadline.argtypes = [u64, i64]
    lib.phip_plan_set_deadline.restype = i32
    lib.phip_plan_cancel.argtypes = [u64]
    lib.phip_plan_cancel.restype = i32
    built, runtime = ctypes.c_int32(0), ctypes.c_int32(0)
    rv = getattr(lib, "phip_runtime_versions", None)  # (absent from round-2 builds used in A/B runs)
    if rv is not None:
        rv.argtypes = [ctypes.POINTER(i32), ctypes.POINTER(i32)]
        rv.restype = i32
    if rv is not None and rv(ctypes.byref(built), ctypes.byref(runtime)) == PHIP_OK and runtime.value > 0:
        if built.value // 10_000_000 != runtime.value // 10_000_000:  # HIP_VERSION = major*1e7 + minor*1e5 + patch
            raise ImportError(f"libpinot_hip.so was built against HIP {built.value} but the process runs HIP "
                              f"{runtime.value} (major versions differ)")
    _lib = lib
    return lib


def check(rc):
    if rc != PHIP_OK:
        raise _ERRORS.get(rc, PhipError)(rc, load().phip_last_error().decode(errors="replace"))
    return rc
