"""Star-tree (StarTreeV2) index writer for test segments, and the ctypes attach of a star-tree to a pinned segment
(ph_segment_add_star_tree).

The writer restates the reference builder so tests can create star-tree segments the way Pinot's segment creation
does (OnHeapSingleTreeBuilder / BaseSingleTreeBuilder, pinot-segment-local/.../startree/v2/builder/
BaseSingleTreeBuilder.java:300-534, OnHeapSingleTreeBuilder.java:66-158; serialisation StarTreeBuilderUtils.java:89-225):

  * raw records sorted by the split-order dimensions' dictIds and merged per distinct dimension tuple
    (sortAndAggregateSegmentRecords; ValueAggregators: COUNT -> LONG count, SUM / MIN / MAX -> DOUBLE);
  * constructStarTree: per node, non-star children = runs of one dictId of the next dimension; a star child (its
    records re-aggregated with that dimension as STAR_IN_FORWARD_INDEX = 0, appended at the end) when the node has
    more than one child and the dimension is not in skipStarNodeCreationForDimensions; children holding more than
    maxLeafRecords records split further;
  * createAggregatedDocs: every node gets an aggregated document (a one-record leaf uses its record; a node with a
    star child uses the star child's);
  * the tree written breadth first, children sorted by dimension value (the star node, -1, first), 7 little-endian
    ints per node after the header (magic, version, header size, dimensions); the dimensions' forward indexes
    fixed-bit packed at the segment column's bit width; the metric pair columns as PASS_THROUGH raw forward indexes.

Children maps are java.util.HashMap<Integer, TreeNode>: the recursion visits them in the map's iteration order
(bucket = key spread & (capacity - 1), insertion order within a bucket), which `_hashmap_order` emulates; it decides
the doc ids of the star-node and aggregated records.  The query side reads whatever tree it is given, so the GPU
parity tests do not depend on this emulation being exact.
"""
import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Sequence

import numpy as np

from . import native as N
from .segment import fixed_bit_pack, num_bits_per_value, write_raw_forward_index

MAGIC = 0xBADDA55B00DAD00D
ALL = -1                   # StarTreeNode.ALL
STAR_IN_FORWARD_INDEX = 0  # StarTreeV2Constants.STAR_IN_FORWARD_INDEX
FUNCTIONS = ("count", "sum", "min", "max")  # AggregationFunctionType.getName() of the supported pairs


@dataclass
class StarTreeBuffers:
    """One star-tree of a segment, as its star_tree_index buffers hold it (StarTreeIndexMapUtils keys)."""
    num_docs: int
    dimensions: List[str]
    pairs: List[str]                      # function-column pair column names, e.g. "count__*", "sum__m"
    tree: np.ndarray                      # the STAR_TREE buffer (OffHeapStarTree format)
    dim_fwd: Dict[str, np.ndarray]        # fixed-bit packed dictIds (parent column's bit width)
    metric_fwd: Dict[str, np.ndarray]     # raw forward indexes (LONG for count__*, DOUBLE otherwise)
    max_leaf_records: int = 10
    skip_star: List[str] = field(default_factory=list)
    # writer-side copies (tests): the star-tree records
    dim_ids: np.ndarray = None            # [num_docs, num_dimensions] int32
    metrics: Dict[str, np.ndarray] = None


def pair_name(function: str, column: str) -> str:
    """AggregationFunctionColumnPair.toColumnName (AggregationFunctionColumnPair.java:51-57): name__column."""
    return f"{function}__{column}"


def _hashmap_order(keys: Sequence[int]) -> List[int]:
    """Iteration order of a java.util.HashMap<Integer, V> filled with `keys` in this order (no removals)."""
    cap = 16
    while len(keys) > cap * 3 // 4:
        cap *= 2
    def bucket(k):
        h = k & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    return [k for _, _, k in sorted((bucket(k), i, k) for i, k in enumerate(keys))]


class _Node:
    __slots__ = ("dim", "value", "start", "end", "agg", "child_dim", "children")

    def __init__(self, dim=-1, value=ALL, start=0, end=0):
        self.dim, self.value, self.start, self.end = dim, value, start, end
        self.agg = -1
        self.child_dim = -1
        self.children = None  # {dictId or ALL: _Node}, insertion order kept


class _Builder:
    def __init__(self, dims: np.ndarray, metrics: List[np.ndarray], kinds: List[str], max_leaf: int, skip: set):
        self.kinds = kinds
        self.max_leaf = max_leaf
        self.skip = skip
        self.nd = dims.shape[1]
        self.D: List[np.ndarray] = []   # star-tree records: dims rows
        self.M: List[list] = []         # metric values rows
        self.num_nodes = 1
        # sortAndAggregateSegmentRecords: stable lexicographic sort, equal tuples merged in doc order
        order = np.lexsort(dims.T[::-1]) if len(dims) else np.zeros(0, np.int64)
        prev = None
        for i in order:
            row = dims[i]
            raw = [None if k == "count" else float(m[i]) for k, m in zip(kinds, metrics)]
            if prev is not None and np.array_equal(row, prev):
                self._apply_raw(self.M[-1], raw)
            else:
                self.D.append(row.copy())
                self.M.append([1 if k == "count" else v for k, v in zip(kinds, raw)])
                prev = row

    def _apply_raw(self, agg, raw):
        for j, k in enumerate(self.kinds):
            if k == "count":
                agg[j] += 1
            elif k == "sum":
                agg[j] = agg[j] + raw[j]
            elif k == "min":
                agg[j] = min(agg[j], raw[j])
            else:
                agg[j] = max(agg[j], raw[j])

    def _merge(self, agg, other):
        if agg is None:
            return list(other)
        for j, k in enumerate(self.kinds):
            if k in ("count", "sum"):
                agg[j] = agg[j] + other[j]
            elif k == "min":
                agg[j] = min(agg[j], other[j])
            else:
                agg[j] = max(agg[j], other[j])
        return agg

    def _new(self, *a):
        self.num_nodes += 1
        return _Node(*a)

    def construct(self, node: _Node, start: int, end: int):
        cd = node.dim + 1
        if cd == self.nd:
            return
        node.child_dim = cd
        children = {}
        s, v = start, int(self.D[start][cd])
        for i in range(start + 1, end):
            x = int(self.D[i][cd])
            if x != v:
                children[v] = self._new(cd, v, s, i)
                s, v = i, x
        children[v] = self._new(cd, v, s, end)
        if cd not in self.skip and len(children) > 1:
            star = self._new(cd, ALL, len(self.D), 0)
            self._star_records(start, end, cd)
            star.end = len(self.D)
            children[ALL] = star
        node.children = children
        for k in _hashmap_order(list(children)):
            ch = children[k]
            if ch.end - ch.start > self.max_leaf:
                self.construct(ch, ch.start, ch.end)

    def _star_records(self, start, end, dim):
        # generateRecordsForStarNode: sort by the dimensions after `dim` (stable), merge equal suffixes
        rows = list(range(start, end))
        rows.sort(key=lambda r: tuple(int(x) for x in self.D[r][dim + 1:]))
        out_d, out_m = [], []
        cur = None
        for r in rows:
            if cur is not None and np.array_equal(self.D[r][dim + 1:], self.D[cur][dim + 1:]):
                out_m[-1] = self._merge(out_m[-1], self.M[r])
            else:
                d = self.D[r].copy()
                d[dim] = STAR_IN_FORWARD_INDEX
                out_d.append(d)
                out_m.append(list(self.M[r]))
                cur = r
        self.D += out_d
        self.M += out_m

    def aggregate(self, node: _Node):
        if node.children is None:
            if node.start == node.end - 1:
                node.agg = node.start
                return list(self.M[node.start])
            agg = None
            for i in range(node.start, node.end):
                agg = self._merge(agg, self.M[i])
            d = self.D[node.start].copy()
            d[node.dim + 1:] = STAR_IN_FORWARD_INDEX
            node.agg = len(self.D)
            self.D.append(d)
            self.M.append(agg)
            return agg
        if ALL in node.children:
            res = None
            for k in _hashmap_order(list(node.children)):
                ch = node.children[k]
                r = self.aggregate(ch)
                if ch.value == ALL:
                    res = r
                    node.agg = ch.agg
            return res
        agg = None
        for k in _hashmap_order(list(node.children)):
            agg = self._merge(agg, self.aggregate(node.children[k]))
        d = self.D[node.children[next(iter(node.children))].start].copy()
        d[node.dim + 1:] = STAR_IN_FORWARD_INDEX
        node.agg = len(self.D)
        self.D.append(d)
        self.M.append(agg)
        return agg

    def serialize(self, root: _Node, names: List[str]) -> np.ndarray:
        head = bytearray()
        hsize = 20 + sum(8 + len(n.encode()) for n in names) + 4
        head += np.array([MAGIC], "<u8").tobytes()
        head += np.array([1, hsize, len(names)], "<i4").tobytes()
        for i, n in enumerate(names):
            b = n.encode()
            head += np.array([i, len(b)], "<i4").tobytes() + b
        head += np.array([self.num_nodes], "<i4").tobytes()
        rows = []
        queue = [root]
        cur = 0
        while queue:
            node = queue.pop(0)
            if node.children is None:
                rows.append([node.dim, node.value, node.start, node.end, node.agg, -1, -1])
            else:
                kids = sorted(node.children.values(), key=lambda c: c.value)
                first = cur + len(queue) + 1
                rows.append([node.dim, node.value, node.start, node.end, node.agg, first, first + len(kids) - 1])
                queue += kids
            cur += 1
        assert cur == self.num_nodes
        return np.frombuffer(bytes(head) + np.array(rows, "<i4").tobytes(), np.uint8).copy()


def build_star_tree(seg, dimensions: Sequence[str], pairs: Sequence[tuple], max_leaf_records: int = 10,
                    skip_star: Sequence[str] = (), values: Dict[str, np.ndarray] = None) -> StarTreeBuffers:
    """A star-tree over `seg` (SegmentBuffers): split order `dimensions` (dictionary columns), function-column
    `pairs` [(function, column)] with function in count / sum / min / max (column "*" for count); `values` holds the
    metric columns' raw values (the writer reads them as PinotSegmentColumnReader.getValue would)."""
    n = seg.num_docs
    dims = np.zeros((n, len(dimensions)), np.int32)
    for j, d in enumerate(dimensions):
        cb = seg.columns[d]
        if cb.raw:
            raise ValueError(f"star-tree dimension {d} has no dictionary")
        dims[:, j] = _dict_ids(cb, n)
    kinds, mets, names = [], [], []
    for fn, col in pairs:
        if fn not in FUNCTIONS:
            raise ValueError(f"unsupported star-tree function {fn}")
        kinds.append(fn)
        names.append(pair_name(fn, col))
        mets.append(None if fn == "count" else np.asarray(values[col], np.float64))
    b = _Builder(dims, mets, kinds, max_leaf_records, {dimensions.index(s) for s in skip_star})
    root = _Node(-1, ALL, 0, len(b.D))
    b.construct(root, 0, len(b.D))
    b.aggregate(root)
    tree = b.serialize(root, list(dimensions))
    D = np.array(b.D, np.int32).reshape(-1, len(dimensions))
    nd = len(D)
    dim_fwd = {d: fixed_bit_pack(D[:, j], seg.columns[d].bits) for j, d in enumerate(dimensions)}
    metrics, metric_fwd = {}, {}
    for j, (nm, k) in enumerate(zip(names, kinds)):
        col = np.array([m[j] for m in b.M], np.int64 if k == "count" else np.float64)
        metrics[nm] = col
        metric_fwd[nm] = write_raw_forward_index(col, "LONG" if k == "count" else "DOUBLE")
    return StarTreeBuffers(nd, list(dimensions), names, tree, dim_fwd, metric_fwd, max_leaf_records, list(skip_star),
                           D, metrics)


def _unpack(fwd: np.ndarray, n: int, bits: int) -> np.ndarray:
    """Fixed-bit unpack of a big-endian MSB-first stream (the writer's own reader; PinotDataBitSet.readInt)."""
    b = np.unpackbits(np.asarray(fwd, np.uint8))[: n * bits].reshape(n, bits).astype(np.int64)
    return (b << np.arange(bits - 1, -1, -1, dtype=np.int64)).sum(axis=1).astype(np.int32)


def _dict_ids(cb, n):
    if cb.is_sorted:
        ids = np.zeros(n, np.int32)
        pairs = np.frombuffer(np.asarray(cb.forward_index, np.uint8).tobytes(), ">i4").reshape(-1, 2)
        for k, (s, e) in enumerate(pairs):
            ids[max(s, 0):e + 1] = k
        return ids
    return _unpack(cb.forward_index, n, cb.bits)


class StarTreeDesc(ctypes.Structure):
    _fields_ = [
        ("tree", ctypes.c_void_p), ("tree_size", ctypes.c_uint64),
        ("num_docs", ctypes.c_int32),
        ("num_dimensions", ctypes.c_int32),
        ("dimensions", ctypes.POINTER(ctypes.c_char_p)),
        ("dimension_forward_index", ctypes.POINTER(ctypes.c_void_p)),
        ("dimension_forward_index_size", ctypes.POINTER(ctypes.c_uint64)),
        ("num_metrics", ctypes.c_int32),
        ("metrics", ctypes.POINTER(ctypes.c_char_p)),
        ("metric_forward_index", ctypes.POINTER(ctypes.c_void_p)),
        ("metric_forward_index_size", ctypes.POINTER(ctypes.c_uint64)),
    ]


def attach(pinned, st: StarTreeBuffers) -> None:
    """ph_segment_add_star_tree: pin the star-tree's buffers beside the segment (StarTreeIndexContainer)."""
    keep = []

    def arr(ctype, items):
        a = (ctype * max(1, len(items)))(*items)
        keep.append(a)
        return a
    tree = np.ascontiguousarray(st.tree, np.uint8)
    dfw = [np.ascontiguousarray(st.dim_fwd[d], np.uint8) for d in st.dimensions]
    mfw = [np.ascontiguousarray(st.metric_fwd[m], np.uint8) for m in st.pairs]
    keep += [tree] + dfw + mfw
    d = StarTreeDesc()
    d.tree, d.tree_size, d.num_docs = tree.ctypes.data, tree.nbytes, st.num_docs
    d.num_dimensions = len(st.dimensions)
    d.dimensions = arr(ctypes.c_char_p, [x.encode() for x in st.dimensions])
    d.dimension_forward_index = arr(ctypes.c_void_p, [a.ctypes.data for a in dfw])
    d.dimension_forward_index_size = arr(ctypes.c_uint64, [a.nbytes for a in dfw])
    d.num_metrics = len(st.pairs)
    d.metrics = arr(ctypes.c_char_p, [x.encode() for x in st.pairs])
    d.metric_forward_index = arr(ctypes.c_void_p, [a.ctypes.data for a in mfw])
    d.metric_forward_index_size = arr(ctypes.c_uint64, [a.nbytes for a in mfw])
    N.check(N.lib().ph_segment_add_star_tree(pinned.handle, ctypes.byref(d)))
