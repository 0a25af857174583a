"""ctypes binding of libpinot_hip.so (include/pinot_hip.h).

The library is built in-tree (``pinot_amd/libpinot_hip.so``, see ``__graft_entry__.build``).  There is no
fallback: if the library is missing or a GPU call fails, the error is raised to the caller.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PH_LIB_PATH") or os.path.join(HERE, "libpinot_hip.so")  # override: kernel experiments

PH_OK = 0
PH_ERR_INVALID_ARGUMENT = 1
PH_ERR_BAD_QUERY = 2
PH_ERR_UNSUPPORTED = 3
PH_ERR_DEVICE = 4
PH_ERR_OUT_OF_MEMORY = 5
PH_ERR_CANCELLED = 6

PH_INT, PH_LONG, PH_FLOAT, PH_DOUBLE, PH_STRING = range(5)
DATA_TYPES = {"INT": PH_INT, "LONG": PH_LONG, "FLOAT": PH_FLOAT, "DOUBLE": PH_DOUBLE, "STRING": PH_STRING}

PH_PRED_EQ, PH_PRED_NOT_EQ, PH_PRED_IN, PH_PRED_NOT_IN, PH_PRED_RANGE = range(5)
PH_FILTER_AND, PH_FILTER_OR, PH_FILTER_NOT, PH_FILTER_PREDICATE = range(4)
PH_AGG_COUNT, PH_AGG_SUM, PH_AGG_MIN, PH_AGG_MAX, PH_AGG_DISTINCTCOUNTHLL = range(5)


class PinotHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class BadQueryError(PinotHipError):
    """BadQueryRequestException (PredicateEvaluatorProvider.java:92-95)."""


class UnsupportedError(PinotHipError):
    """Shape not on the GPU path; the caller falls back to the CPU plan."""


class CancelledError(PinotHipError):
    """Query interrupted or past its end time (QueryException EXECUTION_TIMEOUT / QUERY_CANCELLATION)."""


class ColumnDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data_type", ctypes.c_int32), ("cardinality", ctypes.c_int32),
                ("bits_per_element", ctypes.c_int32), ("is_sorted", ctypes.c_int32),
                ("forward_index", ctypes.c_void_p), ("forward_index_size", ctypes.c_uint64),
                ("dictionary", ctypes.c_void_p), ("dictionary_size", ctypes.c_uint64),
                ("dictionary_entry_size", ctypes.c_int32),
                ("inverted_index", ctypes.c_void_p), ("inverted_index_size", ctypes.c_uint64),
                ("raw_forward_index", ctypes.c_int32),
                ("range_index", ctypes.c_void_p), ("range_index_size", ctypes.c_uint64),
                ("hll_log2m", ctypes.c_int32)]


class MetadataEntry(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char_p), ("value", ctypes.c_char_p)]


class SegmentDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("num_docs", ctypes.c_int32), ("num_columns", ctypes.c_int32),
                ("columns", ctypes.POINTER(ColumnDesc))]


class Predicate(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("column", ctypes.c_char_p), ("num_values", ctypes.c_int32),
                ("values", ctypes.POINTER(ctypes.c_char_p)), ("lower", ctypes.c_char_p),
                ("upper", ctypes.c_char_p), ("lower_inclusive", ctypes.c_int32),
                ("upper_inclusive", ctypes.c_int32)]


class FilterNode(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("num_children", ctypes.c_int32),
                ("children", ctypes.POINTER(ctypes.c_int32)), ("predicate", ctypes.c_int32)]


PH_EXPR_NONE, PH_EXPR_MULT, PH_EXPR_SUB, PH_EXPR_ADD = range(4)
EXPR_CODES = {None: PH_EXPR_NONE, "*": PH_EXPR_MULT, "-": PH_EXPR_SUB, "+": PH_EXPR_ADD}


class Aggregation(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("column", ctypes.c_char_p), ("log2m", ctypes.c_int32),
                ("column2", ctypes.c_char_p), ("expr_op", ctypes.c_int32)]


class OrderBy(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("index", ctypes.c_int32), ("asc", ctypes.c_int32)]


PH_ORDER_GROUP_BY, PH_ORDER_AGGREGATION = 0, 1


class Query(ctypes.Structure):
    _fields_ = [("num_filter_nodes", ctypes.c_int32), ("filter_nodes", ctypes.POINTER(FilterNode)),
                ("filter_root", ctypes.c_int32), ("num_predicates", ctypes.c_int32),
                ("predicates", ctypes.POINTER(Predicate)), ("num_group_by", ctypes.c_int32),
                ("group_by", ctypes.POINTER(ctypes.c_char_p)), ("num_aggregations", ctypes.c_int32),
                ("aggregations", ctypes.POINTER(Aggregation)), ("num_groups_limit", ctypes.c_int64),
                ("end_time_ms", ctypes.c_int64), ("interrupt", ctypes.POINTER(ctypes.c_int32)),
                ("num_order_by", ctypes.c_int32), ("order_by", ctypes.POINTER(OrderBy)), ("limit", ctypes.c_int32),
                ("min_segment_group_trim_size", ctypes.c_int32), ("skip_star_tree", ctypes.c_int32)]


PH_MAX_DENSE_TABLES = 16
PH_REDUCE_SUM_I64, PH_REDUCE_SUM_F64, PH_REDUCE_MIN_I64, PH_REDUCE_MAX_I64, PH_REDUCE_MAX_U32 = range(5)


class DenseLayout(ctypes.Structure):
    _fields_ = [("num_groups", ctypes.c_int64), ("num_tables", ctypes.c_int32),
                ("elems_per_group", ctypes.c_int32 * PH_MAX_DENSE_TABLES),
                ("reduce_op", ctypes.c_int32 * PH_MAX_DENSE_TABLES),
                ("elem_bytes", ctypes.c_int32 * PH_MAX_DENSE_TABLES)]


class ExecStats(ctypes.Structure):
    _fields_ = [("num_docs_scanned", ctypes.c_int64), ("num_entries_scanned_in_filter", ctypes.c_int64),
                ("num_entries_scanned_post_filter", ctypes.c_int64), ("num_total_docs", ctypes.c_int64),
                ("num_segments_processed", ctypes.c_int64), ("num_segments_matched", ctypes.c_int64),
                ("num_groups_limit_reached", ctypes.c_int32), ("sum_precision_flag", ctypes.c_int32),
                ("device_ms", ctypes.c_double), ("host_ms", ctypes.c_double), ("plan_mode", ctypes.c_int32),
                ("limit_pass", ctypes.c_int32),
                ("scan_kernel", ctypes.c_int32), ("num_devices", ctypes.c_int32),
                ("merge_ms", ctypes.c_double), ("finalize_ms", ctypes.c_double), ("scan_ms", ctypes.c_double),
                ("num_segments_star_tree", ctypes.c_int64)]


# every symbol declared in include/pinot_hip.h
EXPORTED_SYMBOLS = (
    "ph_ctx_create", "ph_ctx_create_multi", "ph_ctx_num_devices", "ph_ctx_set_multi_transport", "ph_segment_device", "ph_ctx_destroy",
    "ph_ctx_set_stream", "ph_ctx_set_option", "ph_segment_pin", "ph_segment_check", "ph_segment_load_dir", "ph_filter_execute",
    "ph_segment_unpin",
    "ph_segment_device_bytes", "ph_segment_num_docs", "ph_table_set_dictionary", "ph_table_set_column_type", "ph_query_execute",
    "ph_result_destroy", "ph_result_stats", "ph_result_num_groups", "ph_result_key_entry_size", "ph_result_key_type",
    "ph_result_group_keys", "ph_result_aggregation", "ph_result_key_data", "ph_result_aggregation_data",
    "ph_query_dense_layout", "ph_query_execute_dense", "ph_dense_finalize", "ph_fixed_bit_pack",
    "ph_raw_forward_index_read", "ph_index_map_lookup", "ph_result_datatable", "ph_selftest_unpack",
    "ph_selftest_unpack_staged", "ph_last_error", "ph_version", "ph_segment_add_star_tree", "ph_segment_num_star_trees",
    "ph_star_tree_check",
)

_lib = None


def _share_torch_hip_runtime():
    """One HIP runtime per process.  The PyTorch-ROCm wheel bundles its own libamdhip64 (same SONAME
    libamdhip64.so.7 as /opt/rocm's).  Loaded first, /opt/rocm's copy would make torch load a second runtime
    (with its own HSA runtime) that then finds no GPU; so when torch is installed its copy is loaded first, by
    path and RTLD_GLOBAL, and libpinot_hip.so's NEEDED entry binds to it by SONAME.  Device pointers, streams
    and events are then shared with torch (the multi-GPU combine passes torch tensors to the C-ABI)."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
            return


def lib():
    """Load libpinot_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    _share_torch_hip_runtime()
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "ph_ctx_create": ([i32, ctypes.POINTER(vp)], ctypes.c_int),
        "ph_ctx_create_multi": ([ctypes.POINTER(i32), i32, ctypes.POINTER(vp)], ctypes.c_int),
        "ph_ctx_set_multi_transport": ([vp, i32], ctypes.c_int),
        "ph_ctx_num_devices": ([vp], i32),
        "ph_segment_device": ([vp], i32),
        "ph_ctx_destroy": ([vp], ctypes.c_int),
        "ph_ctx_set_stream": ([vp, vp], ctypes.c_int),
        "ph_ctx_set_option": ([vp, ctypes.c_char_p, i64], ctypes.c_int),
        "ph_segment_pin": ([vp, ctypes.POINTER(SegmentDesc), ctypes.POINTER(vp)], ctypes.c_int),
        "ph_segment_check": ([ctypes.POINTER(SegmentDesc)], ctypes.c_int),
        "ph_segment_unpin": ([vp], ctypes.c_int),
        "ph_segment_load_dir": ([vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), i32, ctypes.POINTER(vp)],
                                ctypes.c_int),
        "ph_segment_device_bytes": ([vp], i64),
        "ph_segment_num_docs": ([vp], i32),
        "ph_table_set_dictionary": ([vp, ctypes.c_char_p, i32, vp, i64, i32], ctypes.c_int),
        "ph_table_set_column_type": ([vp, ctypes.c_char_p, i32], ctypes.c_int),
        "ph_query_execute": ([vp, ctypes.POINTER(Query), ctypes.POINTER(vp), i32, ctypes.POINTER(vp)], ctypes.c_int),
        "ph_filter_execute": ([vp, ctypes.POINTER(Query), vp, vp, ctypes.c_uint64, ctypes.POINTER(ExecStats)],
                              ctypes.c_int),
        "ph_result_destroy": ([vp], ctypes.c_int),
        "ph_result_stats": ([vp, ctypes.POINTER(ExecStats)], ctypes.c_int),
        "ph_result_num_groups": ([vp], i64),
        "ph_result_key_entry_size": ([vp, i32], ctypes.c_int),
        "ph_result_key_type": ([vp, i32], ctypes.c_int),
        "ph_result_group_keys": ([vp, i32, vp], ctypes.c_int),
        "ph_result_aggregation": ([vp, i32, vp], ctypes.c_int),
        "ph_result_key_data": ([vp, i32], vp),
        "ph_result_aggregation_data": ([vp, i32], vp),
        "ph_query_dense_layout": ([vp, ctypes.POINTER(Query), ctypes.POINTER(vp), i32, ctypes.POINTER(DenseLayout)],
                                  ctypes.c_int),
        "ph_query_execute_dense": ([vp, ctypes.POINTER(Query), ctypes.POINTER(vp), i32, ctypes.POINTER(vp),
                                    ctypes.POINTER(ExecStats)], ctypes.c_int),
        "ph_dense_finalize": ([vp, ctypes.POINTER(Query), ctypes.POINTER(vp), i32, ctypes.POINTER(vp), i64, i64,
                               ctypes.POINTER(vp)], ctypes.c_int),
        "ph_fixed_bit_pack": ([vp, i64, i32, vp, ctypes.c_uint64], ctypes.c_int),
        "ph_raw_forward_index_read": ([vp, ctypes.c_uint64, i32, i32, vp], ctypes.c_int),
        "ph_index_map_lookup": ([ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(i64),
                                 ctypes.POINTER(i64)], ctypes.c_int),
        "ph_result_datatable": ([vp, ctypes.POINTER(Query), ctypes.POINTER(MetadataEntry), i32, vp, ctypes.c_uint64,
                                 ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        "ph_selftest_unpack": ([vp, vp, ctypes.c_uint64, i64, i32, vp], ctypes.c_int),
        "ph_selftest_unpack_staged": ([vp, vp, ctypes.c_uint64, i64, i32, i32, vp], ctypes.c_int),
        "ph_segment_add_star_tree": ([vp, vp], ctypes.c_int),
        "ph_segment_num_star_trees": ([vp], i32),
        "ph_star_tree_check": ([vp, ctypes.c_uint64, ctypes.POINTER(i32), ctypes.POINTER(i32)], ctypes.c_int),
        "ph_last_error": ([], ctypes.c_char_p),
        "ph_version": ([], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(code: int):
    if code == PH_OK:
        return
    msg = lib().ph_last_error().decode(errors="replace")
    if code == PH_ERR_BAD_QUERY:
        raise BadQueryError(code, msg)
    if code == PH_ERR_UNSUPPORTED:
        raise UnsupportedError(code, msg)
    if code == PH_ERR_CANCELLED:
        raise CancelledError(code, msg)
    raise PinotHipError(code, msg)
