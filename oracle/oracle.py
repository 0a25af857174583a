"""Python side of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module.  It is the parity checker: it never sits on the product path.

It restates, independently of the product library, the host-side half of the reference path:

* segment creation semantics for dictionary-encoded single-value columns: sorted unique
  dictionary, dictIds by rank, ``bitsPerElement = getNumBitsPerValue(card - 1)``, sortedness
  detection (SegmentColumnarIndexCreator.java:519-541, PinotDataBitSet.java:59-70);
* literal -> dictId mapping of the dictionary-based predicate evaluators
  (EqualsPredicateEvaluatorFactory.java:92-144, NotEqualsPredicateEvaluatorFactory,
  InPredicateEvaluatorFactory.java:158-210, NotInPredicateEvaluatorFactory.java:158-210,
  RangePredicateEvaluatorFactory.SortedDictionaryBasedRangePredicateEvaluator :119-232);
* leaf operator choice and AND/OR simplification (FilterOperatorUtils.java:73-125,
  FilterPlanNode.java:200-318) -- used for numEntriesScannedInFilter;
* table-level value union for group keys (the reference merges on ``Key(Object[] values)``,
  GroupByCombineOperator.java:169-178).

The hot loops (fixed-bit read, scan, group-key generation, aggregation, combine) run in C
(pinot_oracle.c) through ctypes.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _load():
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    lib.or_num_bits_per_value.argtypes = [ctypes.c_int32]
    lib.or_num_bits_per_value.restype = ctypes.c_int
    lib.or_fixed_bit_num_bytes.argtypes = [ctypes.c_int64, ctypes.c_int]
    lib.or_fixed_bit_num_bytes.restype = ctypes.c_int64
    lib.or_fixed_bit_write.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    lib.or_fixed_bit_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
    lib.or_fixed_bit_read.restype = ctypes.c_int32
    lib.or_fixed_bit_read_range.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int32,
                                            ctypes.c_void_p]
    lib.or_murmur_hash_long.argtypes = [ctypes.c_int64]
    lib.or_murmur_hash_long.restype = ctypes.c_int32
    lib.or_murmur_hash_bytes.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32]
    lib.or_murmur_hash_bytes.restype = ctypes.c_int32
    lib.or_hll_cardinality.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.or_hll_cardinality.restype = ctypes.c_int64
    lib.or_execute.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    lib.or_execute.restype = ctypes.c_int
    lib.or_result_free.argtypes = [ctypes.c_void_p]
    return lib


LIB = _load()


class _Column(ctypes.Structure):
    _fields_ = [("cardinality", ctypes.c_int32), ("bits", ctypes.c_int32), ("fwd", ctypes.c_void_p),
                ("sorted", ctypes.c_void_p), ("values", ctypes.c_void_p), ("hash_longs", ctypes.c_void_p),
                ("hash_ints", ctypes.c_void_p), ("global_ids", ctypes.c_void_p)]


class _Segment(ctypes.Structure):
    _fields_ = [("num_docs", ctypes.c_int32), ("num_columns", ctypes.c_int32),
                ("columns", ctypes.POINTER(_Column))]


class _FilterOp(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("arg", ctypes.c_int32), ("match", ctypes.c_void_p),
                ("is_scan", ctypes.c_int32)]


class _Query(ctypes.Structure):
    _fields_ = [("num_filter_ops", ctypes.c_int32), ("filter", ctypes.POINTER(_FilterOp)),
                ("num_group_by", ctypes.c_int32), ("group_cols", ctypes.c_void_p),
                ("group_global_card", ctypes.c_void_p), ("num_aggs", ctypes.c_int32),
                ("agg_fn", ctypes.c_void_p), ("agg_col", ctypes.c_void_p), ("log2m", ctypes.c_int32),
                ("num_groups_limit", ctypes.c_int64), ("agg_col2", ctypes.c_void_p), ("agg_op", ctypes.c_void_p)]


OP_CODES = {None: 0, "*": 1, "-": 2, "+": 3}


def _agg_arrays(q, col_index):
    fn = np.array([AGG_CODES[a.function] for a in q.aggregations], dtype=np.int32)
    col = np.array([col_index[a.column] if a.column else -1 for a in q.aggregations], dtype=np.int32)
    col2 = np.array([col_index[a.column2] if getattr(a, "column2", None) else -1 for a in q.aggregations],
                    dtype=np.int32)
    op = np.array([OP_CODES[getattr(a, "op", None)] for a in q.aggregations], dtype=np.int32)
    return fn, col, col2, op


def _used_columns(q):
    cols = list(q.group_by)
    for a in q.aggregations:
        cols += [c for c in (a.column, getattr(a, "column2", None)) if c]
    if q.filter is not None:
        cols += q.filter.columns()
    return list(dict.fromkeys(cols))


class _Result(ctypes.Structure):
    _fields_ = [("num_groups", ctypes.c_int64), ("keys", ctypes.POINTER(ctypes.c_uint64)),
                ("aggs", ctypes.POINTER(ctypes.c_double)), ("hll", ctypes.POINTER(ctypes.c_uint8)),
                ("num_hll", ctypes.c_int32), ("num_docs_scanned", ctypes.c_int64),
                ("num_entries_scanned_in_filter", ctypes.c_int64),
                ("num_entries_scanned_post_filter", ctypes.c_int64), ("num_total_docs", ctypes.c_int64),
                ("num_groups_limit_reached", ctypes.c_int32)]


OR_F_LEAF, OR_F_AND, OR_F_OR, OR_F_NOT, OR_F_ALL, OR_F_NONE = range(6)
AGG_CODES = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "DISTINCTCOUNTHLL": 4}


# --------------------------------------------------------------------------- codec helpers
def num_bits_per_value(max_value: int) -> int:
    return LIB.or_num_bits_per_value(int(max_value))


def fixed_bit_pack(values: np.ndarray, bits: int) -> np.ndarray:
    values = np.ascontiguousarray(values, dtype=np.int32)
    out = np.zeros(int(LIB.or_fixed_bit_num_bytes(len(values), bits)), dtype=np.uint8)
    LIB.or_fixed_bit_write(values.ctypes.data, len(values), bits, out.ctypes.data)
    return out


def fixed_bit_unpack(buf: np.ndarray, n: int, bits: int, start: int = 0) -> np.ndarray:
    # pad so the reader's look-ahead byte stays in bounds
    b = np.concatenate([np.asarray(buf, dtype=np.uint8), np.zeros(8, np.uint8)])
    out = np.empty(n, dtype=np.int32)
    LIB.or_fixed_bit_read_range(b.ctypes.data, start, bits, n, out.ctypes.data)
    return out


def murmur_hash_long(v: int) -> int:
    return LIB.or_murmur_hash_long(int(v))


def murmur_hash_string(s: str) -> int:
    b = s.encode("utf-8")
    return LIB.or_murmur_hash_bytes(b, len(b), -1)


# --------------------------------------------------------------------------- segments
@dataclass
class OracleColumn:
    name: str
    data_type: str               # INT | LONG | FLOAT | DOUBLE | STRING
    dictionary: np.ndarray       # sorted unique values
    bits: int
    is_sorted: bool
    has_inverted: bool = False
    has_range_index: bool = False  # an exact bit-sliced range index (rangeIndexColumns)
    # a legacy version-1 range index (RangeIndexReaderImpl, inexact) over dictIds: its range starts + the last
    # range's end (inclusive), as RangeIndexCreator's header holds them
    legacy_ranges: Optional[np.ndarray] = None
    # ... over a raw (no-dictionary) column's values: (stored type, range starts + the last range's end as values)
    legacy_raw: Optional[tuple] = None
    fwd: Optional[np.ndarray] = None      # packed big-endian fixed-bit bytes (unsorted)
    sorted_ranges: Optional[np.ndarray] = None  # int32 [card, 2]

    @property
    def cardinality(self) -> int:
        return len(self.dictionary)


@dataclass
class OracleSegment:
    name: str
    num_docs: int
    columns: Dict[str, OracleColumn] = field(default_factory=dict)


def _np_dtype(data_type):
    return {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}.get(data_type)


def build_column(name: str, values: np.ndarray, data_type: str, inverted: bool = False) -> OracleColumn:
    if data_type == "STRING":
        values = np.asarray(values).astype(str)
    else:
        values = np.asarray(values, dtype=_np_dtype(data_type))
    dictionary, dict_ids = np.unique(values, return_inverse=True)
    dict_ids = dict_ids.astype(np.int32).reshape(-1)
    card = len(dictionary)
    bits = num_bits_per_value(card - 1)
    is_sorted = bool(len(dict_ids) == 0 or np.all(dict_ids[1:] >= dict_ids[:-1]))
    col = OracleColumn(name, data_type, dictionary, bits, is_sorted, inverted)
    if is_sorted:
        starts = np.searchsorted(dict_ids, np.arange(card), side="left")
        ends = np.searchsorted(dict_ids, np.arange(card), side="right") - 1
        col.sorted_ranges = np.stack([starts, ends], axis=1).astype(np.int32)
    else:
        col.fwd = fixed_bit_pack(dict_ids, bits)
    return col


def build_segment(name: str, columns: Dict[str, tuple], inverted: Sequence[str] = (),
                  range_index: Sequence[str] = (), legacy_ranges: Optional[Dict[str, np.ndarray]] = None,
                  legacy_raw: Optional[Dict[str, np.ndarray]] = None) -> OracleSegment:
    """columns: name -> (values, data_type); legacy_ranges: name -> a version-1 range index's dictId range starts
    followed by the last range's end"""
    n = None
    seg = OracleSegment(name, 0)
    for c, (vals, dt) in columns.items():
        col = build_column(c, vals, dt, c in inverted)
        col.has_range_index = c in range_index
        if legacy_ranges and c in legacy_ranges:
            col.legacy_ranges = np.asarray(legacy_ranges[c], np.int64)
        if legacy_raw and c in legacy_raw:  # a raw column's version-1 index: its range starts + last end (values)
            col.legacy_raw = (dt, np.asarray(legacy_raw[c]))
        seg.columns[c] = col
        n = len(vals) if n is None else n
        assert n == len(vals)
    seg.num_docs = n or 0
    return seg


def segment_from_dict_ids(name: str, cols: Dict[str, tuple]) -> OracleSegment:
    """Build from (dictionary, dict_ids or packed bytes, data_type, bits) -- used for synthetic bench data.
    cols: name -> dict(dictionary=..., fwd=packed bytes, bits=..., data_type=..., num_docs=...)"""
    seg = OracleSegment(name, 0)
    for c, d in cols.items():
        seg.columns[c] = OracleColumn(c, d["data_type"], d["dictionary"], d["bits"], False, False,
                                      fwd=np.asarray(d["fwd"], dtype=np.uint8))
        seg.num_docs = d["num_docs"]
    return seg


# --------------------------------------------------------------------------- predicate evaluation
def _parse_literal(s: str, data_type: str):
    if data_type in ("INT", "LONG"):
        return int(s)
    if data_type in ("FLOAT", "DOUBLE"):
        return float(s) if data_type == "DOUBLE" else float(np.float32(float(s)))
    return s


def _index_of(d: np.ndarray, v) -> int:
    i = int(np.searchsorted(d, v, side="left"))
    return i if i < len(d) and d[i] == v else -1


def _insertion_index_of(d: np.ndarray, v) -> int:
    """BaseImmutableDictionary.insertionIndexOf: index if found, else -(insertionPoint) - 1."""
    i = int(np.searchsorted(d, v, side="left"))
    if i < len(d) and d[i] == v:
        return i
    return -(i + 1)


def predicate_match(pred, col: OracleColumn):
    """Returns (match bitset over dictIds as uint8, always_true, always_false)."""
    d = col.dictionary
    card = len(d)
    m = np.zeros(card, dtype=np.uint8)
    t = pred.TYPE
    if t == "EQ":
        i = _index_of(d, _parse_literal(pred.value, col.data_type))
        if i < 0:
            return m, False, True
        m[i] = 1
        return m, card == 1, False
    if t == "NOT_EQ":
        i = _index_of(d, _parse_literal(pred.value, col.data_type))
        m[:] = 1
        if i < 0:
            return m, True, False
        m[i] = 0
        return m, False, card == 1
    if t == "IN":
        ids = {_index_of(d, _parse_literal(v, col.data_type)) for v in pred.values} - {-1}
        for i in ids:
            m[i] = 1
        return m, len(ids) == card, len(ids) == 0
    if t == "NOT_IN":
        ids = {_index_of(d, _parse_literal(v, col.data_type)) for v in pred.values} - {-1}
        m[:] = 1
        for i in ids:
            m[i] = 0
        return m, len(ids) == 0, len(ids) == card
    if t == "RANGE":
        if pred.lower == "*":
            start = 0
        else:
            ii = _insertion_index_of(d, _parse_literal(pred.lower, col.data_type))
            start = -(ii + 1) if ii < 0 else (ii if pred.lower_inclusive else ii + 1)
        if pred.upper == "*":
            end = card
        else:
            ii = _insertion_index_of(d, _parse_literal(pred.upper, col.data_type))
            end = -(ii + 1) if ii < 0 else (ii + 1 if pred.upper_inclusive else ii)
        if end - start <= 0:
            return m, False, True
        m[start:end] = 1
        return m, end - start == card, False
    raise ValueError(t)


class _Leaf:
    def __init__(self, kind, col_index=None, match=None, is_scan=False):
        self.kind = kind  # "leaf" | "all" | "none" | "and" | "or" | "not"
        self.col_index = col_index
        self.match = match
        self.is_scan = is_scan
        self.children = []


def raw_inclusive_bounds(p, data_type: str):
    """A raw column's RANGE bounds as its raw-value evaluator holds them (RangePredicateEvaluatorFactory.java:70-92,
    :314-499): unbounded = the type's inclusive min / max (infinities for reals), an exclusive bound moved by one
    (INT wraps at 32 bits) or by Math.nextUp / nextDown (float32 steps for FLOAT)."""
    lu, hu = p.lower == "*", p.upper == "*"
    li, hi_inc = lu or p.lower_inclusive, hu or p.upper_inclusive
    if data_type in ("INT", "LONG"):
        bits = 32 if data_type == "INT" else 64
        mn, mx = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
        wrap = lambda v: ((v - mn) % (1 << bits)) + mn  # noqa: E731
        a = mn if lu else int(p.lower)
        b = mx if hu else int(p.upper)
        return (a if li else wrap(a + 1)), (b if hi_inc else wrap(b - 1))
    f32 = data_type == "FLOAT"
    a = -np.inf if lu else (float(np.float32(float(p.lower))) if f32 else float(p.lower))
    b = np.inf if hu else (float(np.float32(float(p.upper))) if f32 else float(p.upper))
    if not li:
        a = float(np.nextafter(np.float32(a), np.float32(np.inf))) if f32 else float(np.nextafter(a, np.inf))
    if not hi_inc:
        b = float(np.nextafter(np.float32(b), np.float32(-np.inf))) if f32 else float(np.nextafter(b, -np.inf))
    return a, b


def _plan_filter(f, seg: OracleSegment, col_index: Dict[str, int]):
    """FilterPlanNode.constructPhysicalOperator simplification rules."""
    if f.type == "PREDICATE":
        p = f.predicate
        col = seg.columns[p.column]
        match, always_true, always_false = predicate_match(p, col)
        if always_false:
            return _Leaf("none")
        if always_true:
            return _Leaf("all")
        # FilterOperatorUtils.DefaultImplementation.getLeafFilterOperator
        # (FilterOperatorUtils.java:97-120): RANGE -> sorted, else range index, else scan; others -> sorted, else
        # inverted, else an exact range index for EQ (RangeIndexBasedFilterOperator.canEvaluate :56-61), else scan
        if col.is_sorted:
            is_scan, ikind = False, "sorted"
        elif p.TYPE != "RANGE" and col.has_inverted:
            is_scan, ikind = False, "inverted"
        elif col.has_range_index and p.TYPE in ("RANGE", "EQ"):
            is_scan, ikind = False, "range"
        elif (col.legacy_ranges is not None or col.legacy_raw is not None) and p.TYPE == "RANGE":
            # an inexact index evaluates RANGE only (RangeIndexBasedFilterOperator.canEvaluate :56-61): a
            # BitmapDocIdSet of the exact docs, whose entries are the partial ranges' scan (:82-107)
            is_scan, ikind = False, "legacy"
        else:
            is_scan, ikind = True, "scan"
        leaf = _Leaf("leaf", col_index[p.column], match, is_scan)
        leaf.ikind = ikind
        if ikind == "legacy" and col.legacy_raw is not None:
            leaf.raw_bounds = raw_inclusive_bounds(p, col.legacy_raw[0])
        return leaf
    if f.type == "AND":
        kids = []
        for c in f.children:
            k = _plan_filter(c, seg, col_index)
            if k.kind == "none":
                return _Leaf("none")
            if k.kind != "all":
                kids.append(k)
        if not kids:
            return _Leaf("all")
        if len(kids) == 1:
            return kids[0]
        n = _Leaf("and")
        n.children = kids
        return n
    if f.type == "OR":
        kids = []
        for c in f.children:
            k = _plan_filter(c, seg, col_index)
            if k.kind == "all":
                return _Leaf("all")
            if k.kind != "none":
                kids.append(k)
        if not kids:
            return _Leaf("none")
        if len(kids) == 1:
            return kids[0]
        n = _Leaf("or")
        n.children = kids
        return n
    if f.type == "NOT":
        k = _plan_filter(f.children[0], seg, col_index)
        if k.kind == "all":
            return _Leaf("none")
        if k.kind == "none":
            return _Leaf("all")
        n = _Leaf("not")
        n.children = [k]
        return n
    raise ValueError(f.type)


def _merge_same_column(node: _Leaf) -> _Leaf:
    """Same-column scan leaves under one AND / OR become one leaf (their match arrays ANDed / ORed), as the
    reference's query optimizer merges them before planning (MergeEqInFilterOptimizer, MergeRangeFilterOptimizer:
    QueryOptimizer.java:47-49); the statistics then follow the merged tree.  Results are unchanged.  A NOT's child is
    merged too (MergeRangeFilterOptimizer.java:101-103 optimizes NOT operands)."""
    if node.kind == "not":
        node.children = [_merge_same_column(node.children[0])]
        k = node.children[0]
        if k.kind == "all":
            return _Leaf("none")
        if k.kind == "none":
            return _Leaf("all")
        return node
    if node.kind not in ("and", "or"):
        return node
    is_and = node.kind == "and"
    out, first = [], {}
    for k in (_merge_same_column(c) for c in node.children):
        if is_and and k.kind == "leaf" and getattr(k, "ikind", "") == "legacy":
            # MergeRangeFilterOptimizer: ranges of one column under an AND become one RANGE, planned once
            j = first.get(("legacy", k.col_index))
            if j is not None:
                a = out[j]
                out[j] = _Leaf("leaf", a.col_index, (a.match & k.match).astype(a.match.dtype), False)
                out[j].ikind = "legacy"
                if hasattr(a, "raw_bounds"):  # MergeRangeFilterOptimizer: the intersected raw bounds
                    out[j].raw_bounds = (max(a.raw_bounds[0], k.raw_bounds[0]), min(a.raw_bounds[1], k.raw_bounds[1]))
                continue
            first[("legacy", k.col_index)] = len(out)
        if k.kind == "leaf" and k.is_scan:
            j = first.get(k.col_index)
            if j is not None:
                a = out[j]
                m = (a.match & k.match) if is_and else (a.match | k.match)
                out[j] = _Leaf("leaf", a.col_index, m.astype(a.match.dtype), True)
                out[j].ikind = "scan"
                continue
            first[k.col_index] = len(out)
        out.append(k)
    kids = []
    for k in out:
        if k.kind == "leaf" and getattr(k, "ikind", "") == "legacy" and not k.match.any():
            k = _Leaf("none")
        elif k.kind == "leaf" and getattr(k, "ikind", "") == "legacy" and k.match.all():
            k = _Leaf("all")  # the merged RANGE is always true: no range-index leaf
        if k.kind == "leaf" and k.is_scan and not k.match.any():
            k = _Leaf("none")
        elif k.kind == "leaf" and k.is_scan and k.match.all():
            k = _Leaf("all")
        if k.kind == ("none" if is_and else "all"):
            return _Leaf(k.kind)
        if k.kind != ("all" if is_and else "none"):
            kids.append(k)
    if not kids:
        return _Leaf("all" if is_and else "none")
    if len(kids) == 1:
        return kids[0]
    node.children = kids
    return node


def _index_based(k: _Leaf) -> bool:
    """A child whose docIdSet iterator is Sorted- or BitmapBased (AndDocIdSet.java:80-100; an OR of such children
    merges into one bitmap, OrDocIdSet.java:33-52)."""
    if k.kind == "leaf":
        return not k.is_scan
    if k.kind == "or":
        return all(_index_based(c) for c in k.children)
    return False


def _mark_apply_and(node: _Leaf) -> _Leaf:
    """ANDs of index-based children and scan leaves run the scans one after another over the index-based result
    (AndDocIdSet.java:128-170, ScanBasedDocIdIterator.applyAnd): the scans count |D0| + |D0 n S1| + ... entries, not
    numDocs each.  Children are ordered as FilterOperatorUtils.reorderAndFilterChildOperators (:197-241) leaves them
    for the statistic: index-based first, then the scans in query order (every SV scan has SCAN_PRIORITY)."""
    if node.kind == "and":
        idx = [k for k in node.children if _index_based(k)]
        scans = [k for k in node.children if k.kind == "leaf" and k.is_scan]
        if idx and scans and len(idx) + len(scans) == len(node.children) and len(scans) < 256:
            node.children = idx + scans
            node.apply_and = (len(idx), len(scans))
            for k in scans:
                k.counted_by_and = True
            return node
    for c in node.children:
        _mark_apply_and(c)
    return node


def _doc_ids(col: OracleColumn, n: int) -> np.ndarray:
    if col.fwd is not None:
        return fixed_bit_unpack(col.fwd, n, col.bits)
    sr = col.sorted_ranges
    return np.repeat(np.arange(len(sr), dtype=np.int32), (sr[:, 1] - sr[:, 0] + 1).astype(np.int64))


def _eval_docs(node: _Leaf, seg: OracleSegment, used: list) -> np.ndarray:
    n = seg.num_docs
    if node.kind == "leaf":
        return node.match[_doc_ids(seg.columns[used[node.col_index]], n)].astype(bool)
    if node.kind == "all":
        return np.ones(n, bool)
    if node.kind == "none":
        return np.zeros(n, bool)
    kids = [_eval_docs(c, seg, used) for c in node.children]
    if node.kind == "and":
        return np.logical_and.reduce(kids)
    if node.kind == "or":
        return np.logical_or.reduce(kids)
    return ~kids[0]


def and_or_entries(d0: np.ndarray, scans: list, b: np.ndarray, ors: list) -> int:
    """numEntriesScannedInFilter of AndDocIdIterator(RangelessBitmapDocIdIterator(A), OrDocIdIterator(...)) over one
    segment (AndDocIdIterator.java:38-75, OrDocIdIterator.java:73-101, SVScanDocIdIterator.advance :101-112), from
    per-doc booleans: d0 = the merged index-based children, scans = the AND's scan children in order (applyAnd:
    |D0| + |D0 n S1| + ...), b = the OR child, ors = the OR's scan children.  The leapfrog touches the OR at the
    candidates a_i of A with B n [a_(i-1), a_i] non-empty (and a_0); a scan child advances there when it holds no
    doc in [a_(i-1), a_i), examining [a_i, next match] (to the segment end when none, after which it is done)."""
    n = len(d0)
    ent, cur = 0, d0.copy()
    for sc in scans:
        ent += int(cur.sum())
        cur &= sc
    a = np.nonzero(cur)[0]
    if len(a) == 0:
        return ent
    cb = np.concatenate([[0], np.cumsum(b, dtype=np.int64)])  # cb[x] = B docs in [0, x)
    prev = np.concatenate([[a[0]], a[:-1]])
    visited = np.ones(len(a), bool)
    visited[1:] = cb[a[1:] + 1] - cb[prev[1:]] > 0
    for o in ors:
        co = np.concatenate([[0], np.cumsum(o, dtype=np.int64)])
        adv = visited.copy()
        adv[1:] &= co[a[1:]] - co[prev[1:]] > 0
        pos = np.nonzero(o)[0]
        t = a[adv]
        j = np.searchsorted(pos, t)
        hit = j < len(pos)
        ent += int((pos[j[hit]] - t[hit] + 1).sum())
        if not hit.all():
            ent += int(n - t[~hit][0])  # the first advance past the last match scans to the end; the child is done
    return ent


def _filter_plan(f, seg: OracleSegment, col_index: Dict[str, int], used: list):
    """The segment's filter tree for the C program (applyAnd marked; the statistic itself comes from
    filter_entries)."""
    return _mark_apply_and(_merge_same_column(_plan_filter(f, seg, col_index)))


def _emit(node: _Leaf, out: list, keep: list):
    if node.kind == "leaf":
        keep.append(node.match)
        counted = node.is_scan and not getattr(node, "counted_by_and", False)
        out.append((OR_F_LEAF, node.col_index, node.match.ctypes.data, int(counted)))
    elif node.kind == "all":
        out.append((OR_F_ALL, 0, None, 0))
    elif node.kind == "none":
        out.append((OR_F_NONE, 0, None, 0))
    else:
        for c in node.children:
            _emit(c, out, keep)
        code = {"and": OR_F_AND, "or": OR_F_OR, "not": OR_F_NOT}[node.kind]
        ia = getattr(node, "apply_and", None)
        out.append((code, len(node.children), None, (ia[0] << 8 | ia[1]) if ia else 0))


# --------------------------------------------------------------------------- numEntriesScannedInFilter
# A literal simulation of the reference's doc-id iterator tree over one segment, from per-doc booleans: the statistic
# is the sum of the docs every SVScanDocIdIterator examines (SVScanDocIdIterator.java:76-142), which depends on how
# the tree drives it -- next() in 256-doc batches, advance(t) doc by doc from t, applyAnd over the docs it is given.
EOF_DOC = -(1 << 31)  # Constants.EOF (Integer.MIN_VALUE)


class _ScanIt:
    """SVScanDocIdIterator (:54-142)."""
    kind = "scan"

    def __init__(self, match: np.ndarray):
        self.match = match
        self.n = len(match)
        self.pos = np.flatnonzero(match)
        self.next_doc = 0
        self.batch = self.pos[:0]
        self.cursor = 0
        self.first_mismatch = 0
        self.entries = 0

    def next(self):
        if self.cursor >= self.first_mismatch:
            # batches of 256 docs from next_doc until one holds a match (each batch counted whole)
            j = int(np.searchsorted(self.pos, self.next_doc))
            if self.next_doc >= self.n or j == len(self.pos):
                self.entries += max(0, self.n - self.next_doc)
                self.next_doc = max(self.next_doc, self.n)
                self.batch, self.cursor, self.first_mismatch = self.pos[:0], 0, 0
                return EOF_DOC
            d = int(self.pos[j])
            start = self.next_doc + ((d - self.next_doc) // 256) * 256
            end = min(start + 256, self.n)
            self.entries += end - self.next_doc
            self.batch = self.pos[j:int(np.searchsorted(self.pos, end))]
            self.next_doc = end
            self.cursor, self.first_mismatch = 0, len(self.batch)
        d = int(self.batch[self.cursor])
        self.cursor += 1
        return d

    def advance(self, t):
        self.next_doc = t
        self.first_mismatch = 0
        if t >= self.n:
            return EOF_DOC
        j = int(np.searchsorted(self.pos, t))
        if j < len(self.pos):
            d = int(self.pos[j])
            self.entries += d - t + 1
            self.next_doc = d + 1
            return d
        self.entries += self.n - t
        self.next_doc = self.n
        return EOF_DOC

    def apply_and(self, docs: np.ndarray) -> np.ndarray:
        self.entries += int(docs.sum())
        return docs & self.match

    def drain(self):  # next() until EOF: the rest of the batch costs nothing, every later doc is scanned
        self.entries += max(0, self.n - self.next_doc)
        self.next_doc = max(self.next_doc, self.n)
        self.cursor = self.first_mismatch


class _IndexIt:
    """SortedDocIdIterator / BitmapDocIdIterator / RangelessBitmapDocIdIterator: no entries scanned."""

    def __init__(self, docs: np.ndarray, kind: str):
        self.docs = docs
        self.kind = kind  # "sorted" | "bitmap"
        self.pos = np.flatnonzero(docs)
        self.cursor = 0

    def next(self):
        if self.cursor < len(self.pos):
            self.cursor += 1
            return int(self.pos[self.cursor - 1])
        return EOF_DOC

    def advance(self, t):
        self.cursor = max(self.cursor, int(np.searchsorted(self.pos, t)))
        return self.next()

    def drain(self):
        self.cursor = len(self.pos)


class _AndIt:
    """AndDocIdIterator (:38-75)."""
    kind = "and"

    def __init__(self, its):
        self.its = its
        self.next_doc = 0

    def next(self):
        max_doc, max_idx, i, k = self.next_doc, -1, 0, len(self.its)
        while i < k:
            if i == max_idx:
                i += 1
                continue
            d = self.its[i].advance(max_doc)
            if d == EOF_DOC:
                return EOF_DOC
            if d == max_doc:
                i += 1
            else:
                max_doc, max_idx, i = d, i, 0
        self.next_doc = max_doc + 1
        return max_doc

    def advance(self, t):
        self.next_doc = t
        return self.next()

    def drain(self):
        while self.next() != EOF_DOC:
            pass


class _OrIt:
    """OrDocIdIterator (:41-126)."""
    kind = "or"

    def __init__(self, its):
        self.its = list(its)
        self.cur = [-1] * len(its)
        self.live = len(its)
        self.prev = -1

    def _prune(self):
        i = 0
        while i < self.live:
            if self.cur[i] == EOF_DOC:
                self.live -= 1
                self.its[i], self.cur[i] = self.its[self.live], self.cur[self.live]
            else:
                i += 1

    def _step(self, t):
        best, ex = None, False
        for i in range(self.live):
            d = self.cur[i]
            if (t is None and d == self.prev) or (t is not None and d < t):
                d = self.its[i].next() if t is None else self.its[i].advance(t)
                self.cur[i] = d
                if d == EOF_DOC:
                    ex = True
                    continue
            best = d if best is None else min(best, d)
        if ex:
            self._prune()
        if best is None:
            return EOF_DOC
        self.prev = best
        return best

    def next(self):
        return self._step(None)

    def advance(self, t):
        return self._step(t)

    def drain(self):  # every child is driven to EOF by next()
        for i in range(self.live):
            self.its[i].drain()
        self.live = 0


class _NotIt:
    """NotDocIdIterator (:29-70); its constructor already calls the child's next()."""
    kind = "not"

    def __init__(self, child, n):
        self.child, self.n = child, n
        self.next_doc = 0
        c = child.next()
        self.next_non = n if c == EOF_DOC else c

    def next(self):
        while self.next_doc == self.next_non:
            self.next_doc += 1
            c = self.child.next()
            self.next_non = self.n if c == EOF_DOC else c
        if self.next_doc >= self.n:
            return EOF_DOC
        self.next_doc += 1
        return self.next_doc - 1

    def advance(self, t):
        self.next_doc = t
        if t > self.next_non:
            c = self.child.advance(t)
            self.next_non = self.n if c == EOF_DOC else c
        return self.next()

    def drain(self):
        self.child.drain()
        self.next_doc = self.n


def _and_set(makers, n):
    """AndDocIdSet.iterator (AndDocIdSet.java:71-185)."""
    def make():
        its = [m() for m in makers]
        idx = [it for it in its if it.kind in ("sorted", "bitmap")]
        scans = [it for it in its if it.kind == "scan"]
        rest = [it for it in its if it.kind not in ("sorted", "bitmap", "scan")]
        if (idx and scans) or len(idx) > 1:
            docs = np.logical_and.reduce([it.docs for it in idx]) if len(idx) > 1 else idx[0].docs.copy()
            for sc in scans:  # ScanBasedDocIdIterator.applyAnd, in the AND's child order
                docs = sc.apply_and(docs)
            merged = _IndexIt(docs, "bitmap")  # RangelessBitmapDocIdIterator
            return merged if not rest else _AndIt([merged] + rest)
        return _AndIt(its)
    return make


def _or_set(makers, n):
    """OrDocIdSet.iterator (OrDocIdSet.java:61-126)."""
    def make():
        its = [m() for m in makers]
        idx = [it for it in its if it.kind in ("sorted", "bitmap")]
        rest = [it for it in its if it.kind not in ("sorted", "bitmap")]
        if len(idx) > 1:
            merged = _IndexIt(np.logical_or.reduce([it.docs for it in idx]), "bitmap")  # BitmapDocIdIterator
            return merged if not rest else _OrIt([merged] + rest)
        return _OrIt(its)
    return make


_PRIORITY = {"sorted": 0, "bitmap": 100, "range": 200, "legacy": 200, "and": 300, "or": 400, "scan": 500, "inverted": 10000}


def _priority(node: _Leaf) -> int:
    """FilterOperatorUtils.reorderAndFilterChildOperators' priorities (:197-241, PrioritizedFilterOperator): sorted
    0, range index 200, AND 300, OR 400, SV scan 500, NOT its child's; an InvertedIndexFilterOperator is none of the
    listed classes, so UNKNOWN_FILTER_PRIORITY (10000)."""
    if node.kind == "leaf":
        return _PRIORITY[node.ikind]
    if node.kind == "not":
        return _priority(node.children[0])
    return _PRIORITY[node.kind]


def filter_entries(root: _Leaf, seg: OracleSegment, used: list) -> int:
    """numEntriesScannedInFilter of one segment (see filter_entries_of)."""
    return filter_entries_of(root, seg.num_docs, lambda node: _eval_docs(node, seg, used))


def legacy_partial_entries(root: _Leaf, seg: OracleSegment, used: list) -> int:
    """The legacy range-index leaves' scans (RangeIndexBasedFilterOperator.evaluateLegacyRangeFilter :82-107): each
    scans the docs of the ranges holding its bounds -- RangeIndexReaderImpl.findRangeId (:236-243) of the inclusive
    lower and upper dictIds, getPartialMatchesInRange (:300-308; a bound outside every range contributes none, both
    bounds in one range scan it once) -- counted by ScanBasedDocIdIterator.applyAnd (SVScanDocIdIterator.java:115-140).
    Every leaf is evaluated, whatever the tree above it."""
    if root.kind in ("and", "or", "not"):
        return sum(legacy_partial_entries(c, seg, used) for c in root.children)
    if root.kind != "leaf" or getattr(root, "ikind", "") != "legacy":
        return 0
    col = seg.columns[used[root.col_index]]
    if col.legacy_raw is not None:  # over raw values: the predicate's inclusive raw bounds
        lo, hi = root.raw_bounds
        starts, last_end = col.legacy_raw[1][:-1], col.legacy_raw[1][-1]
    else:
        ids = np.flatnonzero(root.match)
        lo, hi = int(ids[0]), int(ids[-1])
        starts, last_end = col.legacy_ranges[:-1], int(col.legacy_ranges[-1])

    def find(v):
        for i, st in enumerate(starts):
            if v < st:
                return i - 1
        return len(starts) - 1 if v <= last_end else len(starts)

    a, b = find(lo), find(hi)
    rids = {r for r in (a, b) if 0 <= r < len(starts)}
    vals = _doc_ids(col, seg.num_docs)
    if col.legacy_raw is not None:  # the docs' raw values (the index ranges hold values, not dictIds)
        vals = col.dictionary[vals]
    total = 0
    for r in rids:
        inside = (vals >= starts[r]) & ((vals < starts[r + 1]) if r + 1 < len(starts) else (vals <= last_end))
        total += int(inside.sum())
    return total


def filter_entries_of(root: _Leaf, n: int, docs_of) -> int:
    """numEntriesScannedInFilter of one segment of n docs: the planned tree's DocIdSets (BaseFilterOperator.getTrues /
    getFalses: NOT swaps them, AND.getFalses = OR of the children's falses, OR.getFalses = AND of them, a leaf's falses
    = NotDocIdSet), the iterator DocIdSetOperator draws from it (:59-86) drained to EOF, summed over the scans.
    docs_of(leaf) = the leaf's per-doc match booleans."""
    scans = []
    if root.kind in ("all", "none"):
        return 0

    def leaf_maker(node):
        docs = docs_of(node)
        if node.ikind == "scan":
            def mk():
                it = _ScanIt(docs)
                scans.append(it)
                return it
            return mk
        kind = "sorted" if node.ikind == "sorted" else "bitmap"
        return lambda: _IndexIt(docs, kind)

    def trues(node):
        if node.kind == "leaf":
            return leaf_maker(node)
        if node.kind == "and":
            kids = sorted(node.children, key=_priority)  # stable, as List.sort
            return _and_set([trues(c) for c in kids], n)
        if node.kind == "or":
            return _or_set([trues(c) for c in node.children], n)
        return falses(node.children[0])

    def falses(node):
        if node.kind == "leaf":
            t = trues(node)
            return lambda: _NotIt(t(), n)
        if node.kind == "and":
            kids = sorted(node.children, key=_priority)
            return _or_set([falses(c) for c in kids], n)
        if node.kind == "or":
            return _and_set([falses(c) for c in node.children], n)
        return trues(node.children[0])

    it = trues(root)()
    it.drain()
    return sum(sc.entries for sc in scans)


# --------------------------------------------------------------------------- execution
@dataclass
class OracleStats:
    num_docs_scanned: int
    num_entries_scanned_in_filter: int
    num_entries_scanned_post_filter: int
    num_total_docs: int
    num_groups_limit_reached: bool


@dataclass
class OracleResult:
    keys: List[tuple]
    aggs: List[list]
    stats: OracleStats


def _hash_arrays(col: OracleColumn):
    if col.data_type in ("INT", "LONG"):
        return col.dictionary.astype(np.int64), None
    if col.data_type == "DOUBLE":
        return col.dictionary.astype(np.float64).view(np.int64), None
    if col.data_type == "FLOAT":
        # clearspring MurmurHash.hash(Object): Float -> hashLong(Float.floatToRawIntBits(f)), the int widened to long
        # (parity unpinned: no reference KAT covers a FLOAT column)
        return col.dictionary.astype(np.float32).view(np.int32).astype(np.int64), None
    if col.data_type == "STRING":
        return None, np.array([murmur_hash_string(s) for s in col.dictionary], dtype=np.int32)
    raise NotImplementedError(f"DISTINCTCOUNTHLL on {col.data_type}")


def execute(q, segments: Sequence[OracleSegment], num_threads: int = 1, filter_stats: bool = True) -> OracleResult:
    """Run a QueryContext over oracle segments; returns groups (value tuples) and intermediate
    aggregation results, plus execution statistics.  filter_stats=False skips the numEntriesScannedInFilter
    iterator simulation (a Python pass: the timed CPU baseline measures the C loop nest only)."""
    keep = []  # keep numpy buffers alive
    used = _used_columns(q)
    col_index = {c: i for i, c in enumerate(used)}

    # table-level value unions for group-by columns
    unions = []
    for g in q.group_by:
        unions.append(np.unique(np.concatenate([s.columns[g].dictionary for s in segments]))
                      if segments else np.array([]))
    log2m = next((a.log2m for a in q.aggregations if a.function == "DISTINCTCOUNTHLL"), 8)

    seg_structs = (_Segment * max(1, len(segments)))()
    filter_programs = []
    extra_entries = []  # per segment: numEntriesScannedInFilter (filter_entries: the iterator simulation)
    for si, s in enumerate(segments):
        cols = (_Column * len(used))()
        keep.append(cols)
        for c, ci in col_index.items():
            oc = s.columns[c]
            cs = cols[ci]
            cs.cardinality = oc.cardinality
            cs.bits = oc.bits
            if oc.fwd is not None:
                fwd = np.concatenate([oc.fwd, np.zeros(8, np.uint8)])
                keep.append(fwd)
                cs.fwd = fwd.ctypes.data
            else:
                sr = np.ascontiguousarray(oc.sorted_ranges, dtype=np.int32)
                keep.append(sr)
                cs.sorted = sr.ctypes.data
            if oc.data_type != "STRING":
                vals = oc.dictionary.astype(np.float64)
                keep.append(vals)
                cs.values = vals.ctypes.data
            if any(a.column == c and a.function == "DISTINCTCOUNTHLL" for a in q.aggregations):
                hl, hi = _hash_arrays(oc)
                if hl is not None:
                    keep.append(hl)
                    cs.hash_longs = hl.ctypes.data
                else:
                    keep.append(hi)
                    cs.hash_ints = hi.ctypes.data
            if c in q.group_by:
                gi = np.searchsorted(unions[q.group_by.index(c)], oc.dictionary).astype(np.int32)
                keep.append(gi)
                cs.global_ids = gi.ctypes.data
        seg_structs[si].num_docs = s.num_docs
        seg_structs[si].num_columns = len(used)
        seg_structs[si].columns = cols
        prog = []
        extra = 0
        if q.filter is not None:
            root = _filter_plan(q.filter, s, col_index, used)
            _emit(root, prog, keep)
            # the statistic from the iterator simulation (the C program's own count is not used)
            if filter_stats:
                merged = _merge_same_column(_plan_filter(q.filter, s, col_index))
                extra = filter_entries(merged, s, used) + legacy_partial_entries(merged, s, used)
        filter_programs.append(prog)
        extra_entries.append(extra)

    stats = [0, 0, 0, 0, False]
    group_cols = np.array([col_index[g] for g in q.group_by], dtype=np.int32)
    gcard = np.array([len(u) for u in unions], dtype=np.int64)
    agg_fn, agg_col, agg_col2, agg_op = _agg_arrays(q, col_index)
    nagg = len(q.aggregations)
    m = 1 << log2m
    hll_idx = [k for k, a in enumerate(q.aggregations) if a.function == "DISTINCTCOUNTHLL"]
    merged_keys: Dict[int, int] = {}
    merged: List[list] = []
    key_list: List[int] = []
    # GroupByOperator.java:114-130 segment group trim: ORDER BY + minSegmentGroupTrimSize > 0 ->
    # GroupByUtils.getTableCapacity(limit, min) = max(5 * limit, min) groups per segment
    seg_trim = int(q.options.get("minSegmentGroupTrimSize", -1)) if hasattr(q, "options") else -1
    trim_size = max(5 * q.limit, seg_trim) if (q.group_by and q.order_by and seg_trim > 0) else None
    if True:
        # one or_execute per segment: each segment has its own dictId-space filter program
        for si in range(len(segments)):
            prog = filter_programs[si]
            ops = (_FilterOp * max(1, len(prog)))()
            for i, (op, arg, ptr, scan) in enumerate(prog):
                ops[i].op, ops[i].arg, ops[i].match, ops[i].is_scan = op, arg, ptr, scan
            qs = _Query(len(prog), ops, len(q.group_by), group_cols.ctypes.data, gcard.ctypes.data, nagg,
                        agg_fn.ctypes.data, agg_col.ctypes.data, log2m, q.num_groups_limit,
                        agg_col2.ctypes.data, agg_op.ctypes.data)
            one = (_Segment * 1)(seg_structs[si])
            res = _Result()
            LIB.or_execute(ctypes.byref(qs), one, 1, 1, ctypes.byref(res))
            keep_rows = None
            if trim_size is not None and res.num_groups > trim_size:
                keep_rows = _segment_trim(res, q, segments[si], unions, nagg, trim_size, hll_idx, log2m)
            _merge(res, q, merged_keys, merged, key_list, nagg, hll_idx, m, keep_rows)
            stats[0] += res.num_docs_scanned
            stats[1] += extra_entries[si]
            stats[2] += res.num_entries_scanned_post_filter
            stats[3] += res.num_total_docs
            stats[4] |= bool(res.num_groups_limit_reached)
            LIB.or_result_free(ctypes.byref(res))
    if not q.group_by and not merged:
        merged.append(_default_row(q, m))
        key_list.append(0)
    keys = []
    for gk in key_list:
        vals = []
        for gi, u in enumerate(unions):
            card = len(u)
            vals.append(_py(u[gk % card]))
            gk //= card
        keys.append(tuple(vals))
    # AggregationPlanNode.java:108-119: no filter, no group-by and only COUNT/MIN/MAX/DISTINCTCOUNTHLL on
    # dictionary columns -> NonScanBasedAggregationOperator (answered from dictionaries / metadata:
    # numDocsScanned = totalDocs, numEntriesScannedPostFilter = 0)
    if q.filter is None and not q.group_by and q.aggregations and all(
            a.function in ("COUNT", "MIN", "MAX", "DISTINCTCOUNTHLL") for a in q.aggregations):
        stats[2] = 0
    return OracleResult(keys, merged, OracleStats(*stats))


def filter_docs(q, seg: OracleSegment):
    """One segment's filter as FilterPlanNode.run's operator yields it (FilterPlanNode.java:83-114): the matching
    docs (bool per doc; BaseFilterOperator.getTrues, :92) and the statistic of its iterator tree
    (BlockDocIdSet.getNumEntriesScannedInFilter, via filter_entries).  No filter: MatchAllFilterOperator."""
    n = seg.num_docs
    if q.filter is None:
        return np.ones(n, bool), 0
    used = _used_columns(q)
    col_index = {c: i for i, c in enumerate(used)}
    merged = _merge_same_column(_plan_filter(q.filter, seg, col_index))
    docs = _eval_docs(merged, seg, used)
    return docs, filter_entries(merged, seg, used) + legacy_partial_entries(merged, seg, used)


def doc_words(mask: np.ndarray) -> np.ndarray:
    """A doc mask as the 64-bit words of ph_filter_execute (bit i of word w = doc 64 w + i)."""
    n = len(mask)
    padded = np.zeros(((n + 63) // 64) * 64, np.uint8)
    padded[:n] = mask
    return np.packbits(padded, bitorder="little").view("<u8").astype(np.uint64)


def execute_timed(q, segments: Sequence[OracleSegment], num_threads: int):
    """Single or_execute call over all segments with a pool of num_threads workers (the timed CPU
    baseline).  All segments must share one filter plan shape (true for the bench workloads)."""
    import time
    keep = []
    used = _used_columns(q)
    col_index = {c: i for i, c in enumerate(used)}
    unions = [np.unique(np.concatenate([s.columns[g].dictionary for s in segments])) for g in q.group_by]
    seg_structs = (_Segment * len(segments))()
    progs = []
    for si, s in enumerate(segments):
        cols = (_Column * len(used))()
        keep.append(cols)
        for c, ci in col_index.items():
            oc = s.columns[c]
            cs = cols[ci]
            cs.cardinality, cs.bits = oc.cardinality, oc.bits
            if oc.fwd is not None:
                fwd = np.concatenate([oc.fwd, np.zeros(8, np.uint8)])
                keep.append(fwd)
                cs.fwd = fwd.ctypes.data
            else:  # sorted column: doc ranges (SortedIndexReaderImpl), as execute()
                sr = np.ascontiguousarray(oc.sorted_ranges, dtype=np.int32)
                keep.append(sr)
                cs.sorted = sr.ctypes.data
            vals = oc.dictionary.astype(np.float64)
            keep.append(vals)
            cs.values = vals.ctypes.data
            if any(a.column == c and a.function == "DISTINCTCOUNTHLL" for a in q.aggregations):
                hl, hi = _hash_arrays(oc)
                keep.append(hl if hl is not None else hi)
                if hl is not None:
                    cs.hash_longs = hl.ctypes.data
                else:
                    cs.hash_ints = hi.ctypes.data
            if c in q.group_by:
                gi = np.searchsorted(unions[q.group_by.index(c)], oc.dictionary).astype(np.int32)
                keep.append(gi)
                cs.global_ids = gi.ctypes.data
        seg_structs[si].num_docs, seg_structs[si].num_columns, seg_structs[si].columns = s.num_docs, len(used), cols
        prog = []
        if q.filter is not None:
            _emit(_mark_apply_and(_merge_same_column(_plan_filter(q.filter, s, col_index))), prog, keep)
        progs.append(prog)
    prog = progs[0]
    ops = (_FilterOp * max(1, len(prog)))()
    for i, (op, arg, ptr, scan) in enumerate(prog):
        ops[i].op, ops[i].arg, ops[i].match, ops[i].is_scan = op, arg, ptr, scan
    group_cols = np.array([col_index[g] for g in q.group_by], dtype=np.int32)
    gcard = np.array([len(u) for u in unions], dtype=np.int64)
    agg_fn, agg_col, agg_col2, agg_op = _agg_arrays(q, col_index)
    log2m = next((a.log2m for a in q.aggregations if a.function == "DISTINCTCOUNTHLL"), 8)
    qs = _Query(len(prog), ops, len(q.group_by), group_cols.ctypes.data, gcard.ctypes.data,
                len(q.aggregations), agg_fn.ctypes.data, agg_col.ctypes.data, log2m, q.num_groups_limit,
                agg_col2.ctypes.data, agg_op.ctypes.data)
    res = _Result()
    t0 = time.perf_counter()
    LIB.or_execute(ctypes.byref(qs), seg_structs, len(segments), num_threads, ctypes.byref(res))
    dt = time.perf_counter() - t0
    n = res.num_groups
    nagg = len(q.aggregations)
    keys = np.ctypeslib.as_array(res.keys, (n,)).copy() if n else np.zeros(0, np.uint64)
    aggs = np.ctypeslib.as_array(res.aggs, (n * max(nagg, 1),)).reshape(n, max(nagg, 1)).copy() if n else None
    LIB.or_result_free(ctypes.byref(res))
    return dt, keys, aggs


def _py(v):
    if isinstance(v, np.generic):
        return v.item()
    return v


def _default_row(q, m):
    row = []
    for a in q.aggregations:
        if a.function == "MIN":
            row.append(float("inf"))
        elif a.function == "MAX":
            row.append(float("-inf"))
        elif a.function == "DISTINCTCOUNTHLL":
            row.append(np.zeros(1 << a.log2m, np.uint8))
        elif a.function == "COUNT":
            row.append(0)
        else:
            row.append(0.0)
    return row


def _java_compare(a, b) -> int:
    """Comparable.compareTo of the boxed ORDER BY values: Long / Integer natural order, Double.compare (NaN
    largest, -0.0 < 0.0), String.compareTo (UTF-16 code-unit order: big-endian UTF-16 bytes compare the same)."""
    if isinstance(a, str) and isinstance(b, str):
        x, y = a.encode("utf-16-be", "surrogatepass"), b.encode("utf-16-be", "surrogatepass")
        return (x > y) - (x < y)
    if isinstance(a, float) or isinstance(b, float):
        a, b = float(a), float(b)
        if a < b:
            return -1
        if a > b:
            return 1
        ka = 0x7ff8000000000000 if a != a else int(np.array(a).view(np.int64))
        kb = 0x7ff8000000000000 if b != b else int(np.array(b).view(np.int64))
        return (ka > kb) - (ka < kb)
    return (a > b) - (a < b)


def _segment_trim(res, q, seg: OracleSegment, unions, nagg, size, hll_idx=(), log2m=8):
    """TableResizer.trimInSegmentResults (TableResizer.java:321-343, makeHeap / downHeap :233-262) over one segment's
    groups fed in ArrayBasedHolder order (ascending raw key over the segment's dictIds, column 0 least significant,
    DictionaryBasedGroupKeyGenerator.java:254-377).  An aggregation's order-by value is its extractFinalResult
    (TableResizer.AggregationFunctionExtractor :425-447): a DISTINCTCOUNTHLL orders by HyperLogLog.cardinality()
    (a long).  Returns the indices of the kept rows of `res`."""
    n = res.num_groups
    m = 1 << log2m
    hll = (np.ctypeslib.as_array(res.hll, (n * len(hll_idx) * m,)).reshape(n, len(hll_idx), m)
           if hll_idx and n else None)
    gkeys = np.ctypeslib.as_array(res.keys, (n,))
    aggs = np.ctypeslib.as_array(res.aggs, (n * max(nagg, 1),)).reshape(n, max(nagg, 1))
    recs = []
    for g in range(n):
        k, raw, mult, vals = int(gkeys[g]), 0, 1, []
        for gi, u in enumerate(unions):
            v = u[k % len(u)]
            k //= len(u)
            d = seg.columns[q.group_by[gi]].dictionary
            raw += int(np.searchsorted(d, v)) * mult
            mult *= len(d)
            vals.append(_py(v))
        ob = []
        for o in q.order_by:
            if o.kind == "aggregation":
                f = q.aggregations[o.ref].function
                if f == "DISTINCTCOUNTHLL":
                    reg = np.ascontiguousarray(hll[g, list(hll_idx).index(o.ref)])
                    ob.append(int(LIB.or_hll_cardinality(reg.ctypes.data, log2m)))
                else:
                    ob.append(int(aggs[g, o.ref]) if f == "COUNT" else float(aggs[g, o.ref]))
            else:
                ob.append(vals[q.group_by.index(o.ref)])
        recs.append((raw, g, ob))
    recs.sort(key=lambda r: r[0])
    asc = [o.asc for o in q.order_by]

    def inter(a, b):  # the intermediate-record comparator
        for i, (x, y) in enumerate(zip(a[2], b[2])):
            c = _java_compare(x, y)
            if not asc[i]:
                c = -c
            if c:
                return c
        return 0

    return set(r[1] for r in table_resizer_heap(recs, inter, size))


def table_resizer_heap(recs, inter, size):
    """TableResizer.trimInSegmentResults' heap (TableResizer.java:233-262,321-343): the first `size` records in
    iterator order heapified under the REVERSED intermediate-record comparator `inter` (makeHeap / downHeap), then
    every later record that compares greater than the top replaces it.  Returns the heap array (index 0 = the
    kept record nearest the trim boundary), as the reference's returned list."""
    def cmp(a, b):  # reversed
        return inter(b, a)

    if len(recs) <= size:
        return list(recs)
    heap = list(recs[:size])

    def down(i):
        e = heap[i]
        while True:
            child = 2 * i + 1
            if child >= size:
                break
            t = heap[child]
            right = child + 1
            if right < size and cmp(heap[right], t) < 0:
                child = right
                t = heap[child]
            if cmp(e, t) <= 0:
                break
            heap[i] = t
            i = child
        heap[i] = e
    i = size >> 1
    while i != 0:
        i -= 1
        down(i)
    for r in recs[size:]:
        if cmp(r, heap[0]) > 0:
            heap[0] = r
            down(0)
    return heap


def _merge(res, q, merged_keys, merged, key_list, nagg, hll_idx, m, keep_rows=None):
    n = res.num_groups
    if n == 0:
        return
    keys = np.ctypeslib.as_array(res.keys, (n,))
    aggs = np.ctypeslib.as_array(res.aggs, (n * max(nagg, 1),)).reshape(n, max(nagg, 1))
    hll = None
    if hll_idx:
        hll = np.ctypeslib.as_array(res.hll, (n * len(hll_idx) * m,)).reshape(n, len(hll_idx), m)
    for g in range(n):
        if keep_rows is not None and g not in keep_rows:
            continue
        k = int(keys[g])
        row = []
        for j, a in enumerate(q.aggregations):
            if a.function == "DISTINCTCOUNTHLL":
                row.append(hll[g, hll_idx.index(j)].copy())
            elif a.function == "COUNT":
                row.append(int(aggs[g, j]))
            else:
                row.append(float(aggs[g, j]))
        if k not in merged_keys:
            merged_keys[k] = len(merged)
            merged.append(row)
            key_list.append(k)
            continue
        dst = merged[merged_keys[k]]
        for j, a in enumerate(q.aggregations):
            f = a.function
            if f in ("COUNT", "SUM"):
                dst[j] = dst[j] + row[j]
            elif f == "MIN":
                dst[j] = min(dst[j], row[j])
            elif f == "MAX":
                dst[j] = max(dst[j], row[j])
            else:
                dst[j] = np.maximum(dst[j], row[j])
