"""Server-side query execution over HBM-pinned segments (ServerQueryExecutorV1Impl for the filter ->
aggregation / group-by shapes), followed by the broker reduce (pinot_amd.reduce).

    ctx = GpuContext(0)
    segs = [ctx.pin(create_segment(...)), ...]
    table = ctx.query("SELECT g, SUM(m) FROM t WHERE f BETWEEN 0 AND 9 GROUP BY g ORDER BY g", segs)

``execute`` returns the combined intermediate results (what GroupByCombineOperator hands to the
broker) and the ExecutionStatistics.  Unsupported shapes raise ``UnsupportedError`` -- the
reference-side plan maker falls back to its CPU plan on that code.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from . import native as N
from .query import (COUNT, DISTINCTCOUNTHLL, MAX, MIN, SUM, FilterContext, QueryContext, parse_sql)
from .reduce import ResultTable, reduce_groups
from .segment import PinnedSegment, SegmentBuffers

_AGG = {COUNT: N.PH_AGG_COUNT, SUM: N.PH_AGG_SUM, MIN: N.PH_AGG_MIN, MAX: N.PH_AGG_MAX,
        DISTINCTCOUNTHLL: N.PH_AGG_DISTINCTCOUNTHLL}
_PRED = {"EQ": N.PH_PRED_EQ, "NOT_EQ": N.PH_PRED_NOT_EQ, "IN": N.PH_PRED_IN, "NOT_IN": N.PH_PRED_NOT_IN,
         "RANGE": N.PH_PRED_RANGE}


@dataclass
class ExecutionStats:
    num_docs_scanned: int
    num_entries_scanned_in_filter: int
    num_entries_scanned_post_filter: int
    num_total_docs: int
    num_segments_processed: int
    num_segments_matched: int
    num_groups_limit_reached: bool
    sum_precision_flag: bool
    device_ms: float
    host_ms: float
    mode: int = 0
    limit_pass: int = 0  # numGroupsLimit: 0 not needed, 1 optimistic scan sufficed, 2 first-seen pass + rescan
    scan_kernel: int = 0  # PH_KERNEL_*: the scan's kernel form (SCAN_KERNEL_NAMES)
    num_devices: int = 0  # multi-device context: devices that scanned segments
    merge_ms: float = 0.0  # multi-device: partial-table combine (RCCL reduce-scatter / local reduce)
    finalize_ms: float = 0.0  # multi-device: merged key shards -> result
    scan_ms: float = 0.0  # multi-device: wall time of the devices' scans into their partial tables
    num_segments_star_tree: int = 0  # segments answered from a star-tree


SCAN_KERNEL_NAMES = {0: "none", 1: "k_scan", 2: "k_agg_lean", 3: "k_agg_sparse", 4: "k_group_lds_lean",
                     5: "k_part_scan + k_part_agg", 6: "k_part_scan2 + k_part_agg",
                     7: "k_scan<MODE_PARTITION> + k_part_agg", 8: "k_part_reg + k_part_agg",
                     9: "k_count_reg",
                     11: "k_group_reg", 12: "k_group_sparse", 14: "k_agg_sparse over roaring containers",
                     15: "k_group_sparse over roaring containers"}


@dataclass
class IntermediateResult:
    """Combined server-side result: columnar group keys and intermediate aggregation results."""
    key_columns: List[object]   # per group-by column: numpy array (numeric) or list of str
    agg_columns: List[np.ndarray]  # per aggregation: int64 (COUNT), float64 (SUM/MIN/MAX), uint8[n, m] (HLL)
    num_groups: int
    functions: List[str]
    stats: ExecutionStats

    @property
    def keys(self) -> List[tuple]:
        if not self.key_columns:
            return [()] * self.num_groups
        cols = [c.tolist() if isinstance(c, np.ndarray) else c for c in self.key_columns]
        return list(zip(*cols))

    @property
    def aggs(self) -> List[list]:
        out = []
        conv = []
        for f, col in zip(self.functions, self.agg_columns):
            if f == COUNT:
                conv.append(col.tolist())
            elif f == DISTINCTCOUNTHLL:
                conv.append(list(col))
            else:
                conv.append(col.tolist())
        for i in range(self.num_groups):
            out.append([c[i] for c in conv])
        return out


def check_plan_supported(q: QueryContext):
    """The plan maker's GPU gate for query options whose reference semantics the GPU path does not reproduce;
    the caller then runs the CPU plan (GpuInstancePlanMaker falls back to InstancePlanMakerImplV2).

    * Segment group trim (GroupByOperator.java:114-130, ORDER BY + ``minSegmentGroupTrimSize`` > 0) runs in the
      library (ph_query.min_segment_group_trim_size): per-segment tables, TableResizer.trimInSegmentResults' heap,
      then the combine (an ORDER BY over DISTINCTCOUNTHLL orders by each group's HyperLogLog.cardinality()).
    * Server trim (IndexedTable.java:63-91, resize when the table exceeds ``groupTrimThreshold``) needs no gate:
      its finish keeps the top records by the same ORDER BY, so the broker's final ORDER BY ... LIMIT over the
      GPU's exact (untrimmed) groups is the same result whenever the reference's own merge is exact."""



class _QueryStruct:
    """Builds the ph_query POD graph and keeps every buffer alive while the call runs.  ``timeoutMs`` (query
    option) becomes the call's end time; ``interrupt`` is a ctypes.c_int32 another thread may set."""

    def __init__(self, q: QueryContext, interrupt=None):
        check_plan_supported(q)
        self.keep = []
        nodes: List[N.FilterNode] = []
        preds: List[N.Predicate] = []

        def s(x):
            b = x.encode()
            self.keep.append(b)
            return b

        def add(f: FilterContext) -> int:
            if f.type == "PREDICATE":
                p = f.predicate
                ps = N.Predicate()
                ps.type = _PRED[p.TYPE]
                ps.column = s(p.column)
                vals = []
                if p.TYPE in ("EQ", "NOT_EQ"):
                    vals = [p.value]
                elif p.TYPE in ("IN", "NOT_IN"):
                    vals = list(p.values)
                else:
                    ps.lower = s(p.lower)
                    ps.upper = s(p.upper)
                    ps.lower_inclusive = int(p.lower_inclusive)
                    ps.upper_inclusive = int(p.upper_inclusive)
                arr = (ctypes.c_char_p * max(1, len(vals)))(*[s(v) for v in vals])
                self.keep.append(arr)
                ps.num_values = len(vals)
                ps.values = arr
                preds.append(ps)
                nodes.append(N.FilterNode(N.PH_FILTER_PREDICATE, 0, None, len(preds) - 1))
                return len(nodes) - 1
            kids = [add(c) for c in f.children]
            arr = (ctypes.c_int32 * max(1, len(kids)))(*kids)
            self.keep.append(arr)
            t = {"AND": N.PH_FILTER_AND, "OR": N.PH_FILTER_OR, "NOT": N.PH_FILTER_NOT}[f.type]
            nodes.append(N.FilterNode(t, len(kids), arr, -1))
            return len(nodes) - 1

        root = add(q.filter) if q.filter is not None else -1
        node_arr = (N.FilterNode * max(1, len(nodes)))(*nodes)
        pred_arr = (N.Predicate * max(1, len(preds)))(*preds)
        gb = (ctypes.c_char_p * max(1, len(q.group_by)))(*[s(g) for g in q.group_by])
        aggs = (N.Aggregation * max(1, len(q.aggregations)))(
            *[N.Aggregation(_AGG[a.function], s(a.column) if a.column else None,
                            a.log2m if a.function == DISTINCTCOUNTHLL else 0,
                            s(a.column2) if a.column2 else None, N.EXPR_CODES[a.op]) for a in q.aggregations])
        self.keep += [node_arr, pred_arr, gb, aggs]
        end_ms = 0
        if "timeoutMs" in q.options:
            import time
            end_ms = int(time.time() * 1000) + int(q.options["timeoutMs"])
        obs = []
        for ob in q.order_by:
            if ob.kind == "aggregation":
                obs.append(N.OrderBy(N.PH_ORDER_AGGREGATION, int(ob.ref), int(ob.asc)))
            elif ob.ref in q.group_by:
                obs.append(N.OrderBy(N.PH_ORDER_GROUP_BY, q.group_by.index(ob.ref), int(ob.asc)))
        ob_arr = (N.OrderBy * max(1, len(obs)))(*obs)
        self.keep.append(ob_arr)
        seg_trim = int(q.options.get("minSegmentGroupTrimSize", -1))
        self.struct = N.Query(len(nodes), node_arr, root, len(preds), pred_arr, len(q.group_by), gb,
                              len(q.aggregations), aggs, q.num_groups_limit, end_ms,
                              ctypes.pointer(interrupt) if interrupt is not None else None,
                              len(obs), ob_arr, int(q.limit), seg_trim,
                              int(str(q.options.get("skipStarTree", "false")).lower() == "true"))


_KEY_DTYPE = {N.PH_INT: np.int32, N.PH_LONG: np.int64, N.PH_FLOAT: np.float32, N.PH_DOUBLE: np.float64}


class _ResultHandle:
    """Owns a ph_result; destroyed when the last IntermediateResult referencing it goes away, or by
    GpuContext.close (a result must not outlive its context: it returns pinned blocks to the context's pool)."""

    def __init__(self, r):
        self.r = r

    def destroy(self):
        if self.r is not None:
            N.lib().ph_result_destroy(self.r)
            self.r = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ph_ctx_set_option names (include/pinot_hip.h).  The library reads no environment; this harness (tests, bench, tools)
# maps PH_<NAME> environment variables onto the options of a context before each of its calls, so a test forces a
# kernel form with monkeypatch.setenv("PH_PART_SETS", "1").
OPTION_NAMES = ("roaring_atomic", "agg_cont", "group_cont", "disable_partition", "lds_table_max", "no_group_cache",
                "group_sparse", "agg_sparse", "tile_words", "limit_eager", "part_generic", "agg_generic",
                "lds_generic", "count_generic", "lds_lean", "group_reg_lg", "stat_fuse", "interrupt_chunks",
                "part_klo", "part_batch_rows", "part_flush_first", "part_depth", "part_lds", "part_sets",
                "part_wg_per_cu", "part_slices", "part_mm_blind", "part_serial", "part_ring_log2", "multi_host_merge",
                "sparse_c")
OPTION_UNSET = -(1 << 63)


class GpuContext:
    """One context per GPU (ph_ctx), or over a set of GPUs of the node (``devices``: ph_ctx_create_multi -- segments
    placed by pinned rows, the devices' partial results merged inside the library; a repeated ordinal is a logical
    shard of that GPU)."""

    TRANSPORTS = {"peer": 0, "rccl": 1}  # PH_TRANSPORT_PEER / PH_TRANSPORT_RCCL

    def __init__(self, device: int = 0, devices=None, transport: str = "peer"):
        import weakref
        h = ctypes.c_void_p()
        if devices is None:
            N.check(N.lib().ph_ctx_create(device, ctypes.byref(h)))
            self.devices = [device]
        else:
            ords = (ctypes.c_int32 * len(devices))(*devices)
            N.check(N.lib().ph_ctx_create_multi(ords, len(devices), ctypes.byref(h)))
            self.devices = list(devices)
            device = devices[0]
            if transport != "peer":  # RCCL communicators are created here, not in the first query
                rc = N.lib().ph_ctx_set_multi_transport(h, self.TRANSPORTS[transport])
                if rc != 0:
                    N.lib().ph_ctx_destroy(h)
                    N.check(rc)
        self.handle = h
        self.device = device
        self._env_options = {}  # options this harness set from PH_* environment variables
        # segments and results of this context: released before it (ph_ctx_destroy contract)
        self._segments = weakref.WeakSet()
        self._results = weakref.WeakSet()

    def close(self):
        if self.handle:
            for r in list(self._results):
                r.destroy()
            for seg in list(self._segments):
                seg.unpin()
            N.lib().ph_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, name: str, value=1):
        """ph_ctx_set_option (None: back to the planner's choice)."""
        N.check(N.lib().ph_ctx_set_option(self.handle, name.encode(), OPTION_UNSET if value is None else int(value)))

    def _sync_env_options(self):
        import os
        want = {}
        for name in OPTION_NAMES:
            v = os.environ.get("PH_" + name.upper())
            if v is not None:
                want[name] = int(v) if v.lstrip("-").isdigit() else 1
        for name in set(self._env_options) | set(want):
            if self._env_options.get(name) != want.get(name):
                self.set_option(name, want.get(name))
        self._env_options = want

    def set_stream(self, stream_ptr: int):
        N.check(N.lib().ph_ctx_set_stream(self.handle, ctypes.c_void_p(stream_ptr)))

    def segment_device(self, seg: PinnedSegment) -> int:
        """Index (into ``devices``) of the device the segment was placed on."""
        return N.lib().ph_segment_device(seg.handle)

    def pin(self, buffers: SegmentBuffers, hll_columns=(), log2m: int = 8) -> PinnedSegment:
        """ph_segment_pin; hll_columns get their DISTINCTCOUNTHLL table (log2m) built at pin."""
        seg = PinnedSegment(self, buffers, hll_columns, log2m)
        self._segments.add(seg)
        return seg

    def load_segment_dir(self, path: str, columns=None) -> PinnedSegment:
        """Pin a segment straight from its on-disk directory (V3 columns.psf or V1 files)."""
        seg = PinnedSegment.from_dir(self, path, columns)
        self._segments.add(seg)
        return seg

    def set_column_type(self, column: str, data_type: str):
        """Schema type of a column (ph_table_set_column_type): what a rank without segments uses for value columns."""
        N.check(N.lib().ph_table_set_column_type(self.handle, column.encode(), N.DATA_TYPES[data_type]))

    def set_schema(self, schema: dict):
        for column, data_type in schema.items():
            self.set_column_type(column, data_type)

    def set_table_dictionary(self, column: str, data_type: str, values: np.ndarray):
        dt = N.DATA_TYPES[data_type]
        if data_type == "STRING":
            enc = [str(v).encode() for v in values]
            width = max([len(e) for e in enc] + [1])
            buf = np.zeros((len(enc), width), np.uint8)
            for i, e in enumerate(enc):
                buf[i, :len(e)] = np.frombuffer(e, np.uint8)
        else:
            buf = np.ascontiguousarray(values, dtype=_KEY_DTYPE[dt])
            width = buf.dtype.itemsize
        N.check(N.lib().ph_table_set_dictionary(self.handle, column.encode(), dt, buf.ctypes.data, len(values), width))

    def execute(self, q: QueryContext, segments: Sequence[PinnedSegment], copy: bool = True,
                interrupt=None) -> IntermediateResult:
        """copy=False returns zero-copy views of the result's pinned columns; they stay valid while the
        returned IntermediateResult is alive.  ``interrupt``: optional ctypes.c_int32; setting it non-zero from
        another thread cancels the call (CancelledError)."""
        self._sync_env_options()
        qs = _QueryStruct(q, interrupt)
        segs = (ctypes.c_void_p * max(1, len(segments)))(*[s.handle for s in segments])
        r = ctypes.c_void_p()
        N.check(N.lib().ph_query_execute(self.handle, ctypes.byref(qs.struct), segs, len(segments), ctypes.byref(r)))
        handle = _ResultHandle(r)
        self._results.add(handle)
        res = self._read_result(q, r, copy)
        if not copy:
            res._handle = handle
        return res

    def execute_datatable(self, q: QueryContext, segments: Sequence[PinnedSegment], extra=None) -> bytes:
        """The query's server response: ph_query_execute then ph_result_datatable (DataTable V4 bytes, as
        InstanceResponseBlock.toDataTable).  ``extra``: metadata entries appended to the results metadata."""
        self._sync_env_options()
        qs = _QueryStruct(q)
        segs = (ctypes.c_void_p * max(1, len(segments)))(*[s.handle for s in segments])
        r = ctypes.c_void_p()
        L = N.lib()
        N.check(L.ph_query_execute(self.handle, ctypes.byref(qs.struct), segs, len(segments), ctypes.byref(r)))
        try:
            items = list((extra or {}).items())
            keep = [(k.encode(), str(v).encode()) for k, v in items]
            ents = (N.MetadataEntry * max(1, len(keep)))(*[N.MetadataEntry(k, v) for k, v in keep])
            size = ctypes.c_uint64()
            N.check(L.ph_result_datatable(r, ctypes.byref(qs.struct), ents, len(keep), None, 0, ctypes.byref(size)))
            buf = (ctypes.c_uint8 * size.value)()
            N.check(L.ph_result_datatable(r, ctypes.byref(qs.struct), ents, len(keep), buf, size.value,
                                          ctypes.byref(size)))
            return bytes(buf)
        finally:
            L.ph_result_destroy(r)

    @staticmethod
    def _read_result(q: QueryContext, r, copy: bool = True) -> IntermediateResult:
        L = N.lib()
        st = N.ExecStats()
        N.check(L.ph_result_stats(r, ctypes.byref(st)))
        n = L.ph_result_num_groups(r)
        def view(ptr, nbytes):
            if not nbytes:
                return np.zeros(0, np.uint8)
            a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (nbytes,))
            return a.copy() if copy else a

        key_cols = []
        for g in range(len(q.group_by)):
            es = L.ph_result_key_entry_size(r, g)
            raw = view(L.ph_result_key_data(r, g), n * es)
            t = L.ph_result_key_type(r, g)
            if t == N.PH_STRING:
                # fixed-width NUL-padded entries: numpy's bytes dtype drops the padding, one vectorised UTF-8 decode
                m = np.ascontiguousarray(raw[:n * es]).view(f"S{es}") if n else np.zeros(0, "S1")
                key_cols.append(np.char.decode(m, "utf-8").tolist())
            else:
                key_cols.append(raw.view(_KEY_DTYPE[t]))
        agg_cols = []
        for k, a in enumerate(q.aggregations):
            if a.function == DISTINCTCOUNTHLL:
                arr = view(L.ph_result_aggregation_data(r, k), n << a.log2m).reshape(n, 1 << a.log2m)
            elif a.function == COUNT:
                arr = view(L.ph_result_aggregation_data(r, k), 8 * n).view(np.int64)
            else:
                arr = view(L.ph_result_aggregation_data(r, k), 8 * n).view(np.float64)
            agg_cols.append(arr)
        stats = ExecutionStats(st.num_docs_scanned, st.num_entries_scanned_in_filter,
                               st.num_entries_scanned_post_filter, st.num_total_docs, st.num_segments_processed,
                               st.num_segments_matched, bool(st.num_groups_limit_reached),
                               bool(st.sum_precision_flag), st.device_ms, st.host_ms, st.plan_mode,
                               st.limit_pass, st.scan_kernel, st.num_devices, st.merge_ms, st.finalize_ms,
                               st.scan_ms, st.num_segments_star_tree)
        return IntermediateResult(key_cols, agg_cols, n, [a.function for a in q.aggregations], stats)

    # ---------------------------------------------------------------- segment-level filter (plug point 2)
    def filter(self, sql_or_q, segment: PinnedSegment, words: bool = True):
        """ph_filter_execute: one segment's WHERE clause on the GPU -- what a GpuFilterOperator returns from
        getTrues() (BaseFilterOperator.java:92).  Returns (doc-bitmap words as uint64 -- bit i of word w is doc
        64 w + i -- or None when ``words`` is False, matching-doc count, ExecutionStats)."""
        q = parse_sql(sql_or_q) if isinstance(sql_or_q, str) else sql_or_q
        self._sync_env_options()
        qs = _QueryStruct(q)
        nd = segment.num_docs
        out = np.zeros(max(1, (nd + 63) // 64), np.uint64) if words else None
        st = N.ExecStats()
        N.check(N.lib().ph_filter_execute(self.handle, ctypes.byref(qs.struct), segment.handle,
                                          out.ctypes.data if words else None, out.size if words else 0,
                                          ctypes.byref(st)))
        stats = ExecutionStats(st.num_docs_scanned, st.num_entries_scanned_in_filter,
                               st.num_entries_scanned_post_filter, st.num_total_docs, st.num_segments_processed,
                               st.num_segments_matched, bool(st.num_groups_limit_reached),
                               bool(st.sum_precision_flag), st.device_ms, st.host_ms, st.plan_mode,
                               st.limit_pass, st.scan_kernel, st.num_devices, st.merge_ms, st.finalize_ms,
                               st.scan_ms, st.num_segments_star_tree)
        if words:
            out = out[:(nd + 63) // 64]
        return out, int(st.num_docs_scanned), stats

    # ---------------------------------------------------------------- dense partials (multi-GPU combine)
    def dense_layout(self, q: QueryContext, segments: Sequence[PinnedSegment]) -> N.DenseLayout:
        """ph_query_dense_layout: the dense partial tables of ``q`` (count, element type, reduce op)."""
        self._sync_env_options()
        qs = _QueryStruct(q)
        segs = (ctypes.c_void_p * max(1, len(segments)))(*[s.handle for s in segments])
        lay = N.DenseLayout()
        N.check(N.lib().ph_query_dense_layout(self.handle, ctypes.byref(qs.struct), segs, len(segments),
                                              ctypes.byref(lay)))
        return lay

    def execute_dense(self, q: QueryContext, segments: Sequence[PinnedSegment], table_ptrs: Sequence[int]):
        """ph_query_execute_dense into caller-owned device tables (device pointers, layout order)."""
        self._sync_env_options()
        qs = _QueryStruct(q)
        segs = (ctypes.c_void_p * max(1, len(segments)))(*[s.handle for s in segments])
        tabs = (ctypes.c_void_p * max(1, len(table_ptrs)))(*table_ptrs)
        st = N.ExecStats()
        N.check(N.lib().ph_query_execute_dense(self.handle, ctypes.byref(qs.struct), segs, len(segments), tabs,
                                               ctypes.byref(st)))
        return st

    def dense_finalize(self, q: QueryContext, segments: Sequence[PinnedSegment], table_ptrs: Sequence[int],
                       group_begin: int, group_end: int, copy: bool = True) -> IntermediateResult:
        """ph_dense_finalize of key shard [group_begin, group_end) (pointers to the shard's first group)."""
        self._sync_env_options()
        qs = _QueryStruct(q)
        segs = (ctypes.c_void_p * max(1, len(segments)))(*[s.handle for s in segments])
        tabs = (ctypes.c_void_p * max(1, len(table_ptrs)))(*table_ptrs)
        r = ctypes.c_void_p()
        N.check(N.lib().ph_dense_finalize(self.handle, ctypes.byref(qs.struct), segs, len(segments), tabs,
                                          group_begin, group_end, ctypes.byref(r)))
        handle = _ResultHandle(r)
        self._results.add(handle)
        res = self._read_result(q, r, copy)
        if not copy:
            res._handle = handle
        return res

    def query(self, sql_or_q, segments: Sequence[PinnedSegment]) -> ResultTable:
        q = parse_sql(sql_or_q) if isinstance(sql_or_q, str) else sql_or_q
        r = self.execute(q, segments)
        return reduce_groups(q, r.keys, r.aggs)
