"""TEST INFRASTRUCTURE ONLY -- the CPU oracle's restatement of the reference's star-tree query path.  Imported by tests
only; nothing under pinot_amd/ uses it.  Parity pin: the parse is checked against the reference's own star-tree index
(pinot-segment-local/src/test/resources/data/startree/segment/star_tree_index + its metadata.properties), committed
as tests/golden/startree_segment/; the traversal and the aggregation over star-tree records are restated from:

  OffHeapStarTree / OffHeapStarTreeNode     pinot-segment-local/.../startree/OffHeapStarTree.java:45-83,
                                            OffHeapStarTreeNode.java:29-158 (7 little-endian ints per node)
  StarTreeUtils                             pinot-core/.../startree/StarTreeUtils.java:56-282 (function-column
                                            pairs, predicate evaluators per column, isFitForStarTree)
  StarTreeFilterOperator                    pinot-core/.../startree/operator/StarTreeFilterOperator.java:157-443
                                            (BFS traversal, remaining predicate columns, the AND it builds)
  GroupByPlanNode / AggregationPlanNode     GroupByPlanNode.java:77-99, AggregationPlanNode.java:100-141 (when the
                                            star-tree serves a segment; fast count / metadata plans come first)
  StarTreeProjectPlanNode                   StarTreeProjectPlanNode.java:60-88 (projected columns = pair columns +
                                            group-by columns)
  CountAggregationFunction / Sum / Min / Max over the pair columns (COUNT sums count__*)
"""
import struct
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from . import oracle as O

MAGIC = 0xBADDA55B00DAD00D
ALL = -1


@dataclass
class _F:
    """A filter node (FilterContext shape: type, children, predicate)."""
    type: str
    children: tuple = ()
    predicate: object = None


@dataclass
class Tree:
    dimensions: List[str]
    nodes: np.ndarray  # [num_nodes, 7]: dim, value, start, end, aggregated doc, first child, last child


def parse_tree(buf: bytes) -> Tree:
    """OffHeapStarTree(PinotDataBuffer) (OffHeapStarTree.java:45-83): magic, version, root offset (= header size),
    dimension names (id, length, UTF-8), node count; then the nodes, breadth first."""
    b = bytes(buf)
    magic, version, root, nd = struct.unpack_from("<QiiI", b, 0)
    if magic != MAGIC or version != 1:
        raise ValueError("not a star-tree buffer")
    off = 20
    names = [None] * nd
    for _ in range(nd):
        i, ln = struct.unpack_from("<ii", b, off)
        off += 8
        names[i] = b[off:off + ln].decode("utf-8")
        off += ln
    (num_nodes,) = struct.unpack_from("<i", b, off)
    off += 4
    if off != root or off + 28 * num_nodes != len(b):
        raise ValueError("star-tree header / size mismatch")
    nodes = np.frombuffer(b, "<i4", count=7 * num_nodes, offset=root).reshape(num_nodes, 7).astype(np.int64)
    return Tree(names, nodes)


def _java_string_hash(s: str) -> int:
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h


def java_hashset_order(names: List[str]) -> List[str]:
    """Iteration order of a java.util.HashSet<String> of < 13 names (capacity 16): bucket (hash ^ hash >>> 16) & 15,
    insertion order within a bucket."""
    def bucket(s):
        h = _java_string_hash(s)
        return (h ^ (h >> 16)) & 15
    return [s for _, _, s in sorted((bucket(s), i, s) for i, s in enumerate(names))]


def predicate_evaluators(filt, seg: "O.OracleSegment"):
    """StarTreeUtils.extractPredicateEvaluatorsMap (:85-134) + isOrClauseValidForStarTree (:179-214): column ->
    [composite = list of predicates ORed], in BFS order; None when the filter cannot be solved by the star-tree.
    Always-true predicates drop out, an always-true OR drops out whole."""
    out: Dict[str, list] = {}
    if filt is None:
        return out
    queue = [filt]
    while queue:
        f = queue.pop(0)
        if f.type == "AND":
            queue.extend(f.children)
        elif f.type == "NOT":
            return None
        elif f.type == "OR":
            preds = []
            if not _or_predicates(f, preds):
                return None
            col, evs, always_true = None, [], False
            for p in preds:
                m, at, af = O.predicate_match(p, seg.columns[p.column])
                if at:
                    always_true = True
                    break
                if not af:
                    if col is None:
                        col = p.column
                    elif col != p.column:
                        return None
                    evs.append((p, m))
            if always_true or not evs:
                # (an OR of only always-false predicates keeps an empty list: always true there too, NOTE :107)
                continue
            out.setdefault(col, []).append(evs)
        else:
            p = f.predicate
            m, at, af = O.predicate_match(p, seg.columns[p.column])
            if not at:
                out.setdefault(p.column, []).append([(p, m)])
    return out


def _or_predicates(f, preds) -> bool:
    for c in f.children:
        if c.type in ("AND", "NOT"):
            return False
        if c.type == "OR":
            if not _or_predicates(c, preds):
                return False
        else:
            preds.append(c.predicate)
    return True


def _matching_ids(composites) -> Optional[set]:
    """getMatchingDictIds (:375-443): the AND of the column's composites (each an OR of its predicates' ids), the
    first composite by priority EQ < IN < RANGE < NOT_EQ / NOT_IN < OR (the set is the same in any order)."""
    ids = None
    for comp in composites:
        s = set()
        for _, m in comp:
            s |= set(np.nonzero(m)[0].tolist())
        ids = s if ids is None else ids & s
    return ids


def traverse(tree: Tree, evals: Dict[str, list], group_by: List[str]):
    """StarTreeFilterOperator.traverseStarTree (:207-358): (matched star-tree docs as a sorted array, remaining
    predicate columns in their HashSet order) or None (a predicate column matches no dictId)."""
    nodes = tree.nodes
    dims = tree.dimensions
    matched = []
    root = 0

    def leaf(i):
        return nodes[i, 5] == -1

    found_leaf = leaf(root)
    # remainingPredicateColumns = new HashSet<>(map.keySet()): iteration order only matters for the final copy
    remaining = list(evals.keys())
    remaining_gb = set(group_by)
    global_remaining = list(remaining) if found_leaf else None
    queue = [root]
    cur_dim = -1
    matching = None
    while queue:
        i = queue.pop(0)
        dim = int(nodes[i, 0])
        if dim > cur_dim:
            name = dims[dim]
            if name in remaining:
                remaining.remove(name)
            remaining_gb.discard(name)
            if found_leaf and global_remaining is None:
                global_remaining = list(remaining)
            matching = None
            cur_dim = dim
        if not remaining and not remaining_gb:
            matched.append((int(nodes[i, 4]), int(nodes[i, 4]) + 1))
            continue
        if leaf(i):
            matched.append((int(nodes[i, 2]), int(nodes[i, 3])))
            continue
        child_dim = dims[dim + 1]
        first, last = int(nodes[i, 5]), int(nodes[i, 6])
        star = None
        if (global_remaining is None or child_dim not in global_remaining) and child_dim not in remaining_gb:
            if nodes[first, 1] == ALL:
                star = first
        if child_dim in remaining:
            if matching is None:
                matching = _matching_ids(evals[child_dim])
                if not matching:
                    return None
            nm = len(matching)
            nch = last - first + 1
            if nm * 10 > nch:
                if star is not None and nm >= nch - 1:
                    kids = [c for c in range(first, last + 1) if int(nodes[c, 1]) in matching]
                    if len(kids) == nch - 1:
                        queue.append(star)
                        found_leaf |= leaf(star)
                    else:
                        queue += kids
                        found_leaf |= any(leaf(c) for c in kids)
                else:
                    for c in range(first, last + 1):
                        if int(nodes[c, 1]) in matching:
                            queue.append(c)
                            found_leaf |= leaf(c)
            else:
                # IntOpenHashSet iteration order does not change the matched set
                vals = nodes[first:last + 1, 1]
                for v in sorted(matching):
                    k = np.searchsorted(vals, v)
                    if k < len(vals) and vals[k] == v:
                        queue.append(first + int(k))
                        found_leaf |= leaf(first + int(k))
        else:
            if star is not None:
                queue.append(star)
                found_leaf |= leaf(star)
            else:
                for c in range(first, last + 1):
                    if nodes[c, 1] != ALL:
                        queue.append(c)
                        found_leaf |= leaf(c)
    docs = np.zeros(0, np.int64)
    if matched:
        docs = np.unique(np.concatenate([np.arange(a, b) for a, b in matched]))
    rem = java_hashset_order([c for c in evals if c in (global_remaining or [])])
    return docs, rem


@dataclass
class StarTreeData:
    """One star-tree of an oracle segment: the tree and its records (dictIds of the split-order dimensions, pair
    column values)."""
    tree: Tree
    num_docs: int
    dim_ids: Dict[str, np.ndarray]
    metrics: Dict[str, np.ndarray]


def from_buffers(tree_bytes, num_docs: int, dim_fwd: Dict[str, np.ndarray], bits: Dict[str, int],
                 metric_values: Dict[str, np.ndarray]) -> StarTreeData:
    t = parse_tree(tree_bytes)
    ids = {d: O.fixed_bit_unpack(np.asarray(dim_fwd[d], np.uint8), num_docs, bits[d]).astype(np.int64)
           for d in t.dimensions}
    return StarTreeData(t, num_docs, ids, {k: np.asarray(v) for k, v in metric_values.items()})


PAIR = {"COUNT": "count", "SUM": "sum", "MIN": "min", "MAX": "max"}


def pairs_of(q) -> Optional[List[str]]:
    """StarTreeUtils.extractAggregationFunctionPairs (:56-71): None when an aggregation is not a plain column (or *)
    of a supported function."""
    out = []
    for a in q.aggregations:
        if a.function not in PAIR or getattr(a, "op", None) or getattr(a, "column2", None):
            return None
        out.append(f"{PAIR[a.function]}__{a.column if a.column else '*'}")
    return out


def fit(q, seg, st: StarTreeData):
    """(pairs, evaluators) when the segment's plan node takes the star-tree (skipStarTree unset, every pair present,
    predicate and group-by columns all dimensions), else None."""
    if str(q.options.get("skipStarTree", "false")).lower() == "true":
        return None
    pairs = pairs_of(q)
    if pairs is None or any(p not in st.metrics for p in pairs):
        return None
    evals = predicate_evaluators(q.filter, seg)
    if evals is None:
        return None
    dims = set(st.tree.dimensions)
    if not set(q.group_by) <= dims or not set(evals) <= dims:
        return None
    return pairs, evals


def execute(q, seg, st: StarTreeData, pairs, evals):
    """One segment through the star-tree: {group key tuple: [aggregation values]} and the segment's statistics
    (numDocsScanned, numEntriesScannedInFilter, numEntriesScannedPostFilter, numTotalDocs)."""
    tr = traverse(st.tree, evals, q.group_by)
    nproj = len(set(pairs) | set(q.group_by))
    if tr is None:
        return {}, (0, 0, 0, seg.num_docs)
    d0, rem = tr
    # the AND StarTreeFilterOperator builds (:165-198): [BitmapBasedFilterOperator of d0] + per remaining column (its
    # HashSet order) one operator per composite -- a scan leaf, or an OR of scan leaves -- over the star-tree's
    # dimension columns (forward index + dictionary only: scans), through FilterOperatorUtils.getAndFilterOperator
    # (priorities: bitmap 100, OR 400, scan 500; stable), after the query optimizer's same-column merges
    view = O.OracleSegment("startree", st.num_docs)
    for d in st.tree.dimensions:
        pc = seg.columns[d]
        view.columns[d] = O.OracleColumn(d, pc.data_type, pc.dictionary, pc.bits, False,
                                         fwd=O.fixed_bit_pack(st.dim_ids[d].astype(np.int64), pc.bits))
    used = list(rem)
    col_index = {c: i for i, c in enumerate(used)}
    comps = []
    for col in rem:
        for comp in evals[col]:
            leaves = [_F("PREDICATE", (), p) for p, _ in comp]
            comps.append(leaves[0] if len(leaves) == 1 else _F("OR", tuple(leaves)))
    mask = np.zeros(st.num_docs, bool)
    mask[d0] = True
    entries = 0
    if comps:
        rest = O._merge_same_column(O._plan_filter(_F("AND", tuple(comps)), view, col_index))
        if rest.kind == "none":
            mask[:] = False
        elif rest.kind != "all":
            mask &= O._eval_docs(rest, view, used)
            root = O._Leaf("and")
            b0 = O._Leaf("leaf")
            b0.ikind, b0.docs = "bitmap", np.isin(np.arange(st.num_docs), d0)
            root.children = [b0] + (rest.children if rest.kind == "and" else [rest])
            entries = O.filter_entries_of(
                root, st.num_docs, lambda nd: nd.docs if hasattr(nd, "docs") else O._eval_docs(nd, view, used))
    docs = np.nonzero(mask)[0]
    groups: Dict[tuple, list] = {}
    gids = [st.dim_ids[g] for g in q.group_by]
    for d in docs:
        key = tuple(O._py(seg.columns[g].dictionary[int(gids[k][d])]) for k, g in enumerate(q.group_by))
        row = groups.get(key)
        if row is None:
            row = [None] * len(pairs)
            groups[key] = row
        for j, (a, p) in enumerate(zip(q.aggregations, pairs)):
            v = st.metrics[p][d]
            if a.function == "COUNT":
                row[j] = (row[j] or 0) + int(v)
            elif a.function == "SUM":
                row[j] = (row[j] or 0.0) + float(v)
            elif a.function == "MIN":
                row[j] = float(v) if row[j] is None else min(row[j], float(v))
            else:
                row[j] = float(v) if row[j] is None else max(row[j], float(v))
    return groups, (len(docs), int(entries), len(docs) * nproj, seg.num_docs)


def execute_with_star_trees(q, segments):
    """A query over [(OracleSegment, StarTreeData or None)]: each segment through its star-tree when the plan node
    takes it (fit), else through oracle.execute; per-group results merged as the combine does (COUNT / SUM add, MIN /
    MAX), statistics summed.  Returns (keys, aggs, stats dict, segments served by a star-tree)."""
    merged: Dict[tuple, list] = {}
    order: List[tuple] = []
    stats = dict(num_docs_scanned=0, num_entries_scanned_in_filter=0, num_entries_scanned_post_filter=0,
                 num_total_docs=0)
    served = 0

    def fold(key, row):
        cur = merged.get(key)
        if cur is None:
            merged[key] = list(row)
            order.append(key)
            return
        for j, a in enumerate(q.aggregations):
            if row[j] is None:
                continue
            if cur[j] is None:
                cur[j] = row[j]
            elif a.function in ("COUNT", "SUM"):
                cur[j] = cur[j] + row[j]
            elif a.function == "MIN":
                cur[j] = min(cur[j], row[j])
            else:
                cur[j] = max(cur[j], row[j])
    for seg, st in segments:
        f = fit(q, seg, st) if st is not None else None
        if q.group_by == [] and f is not None:
            # AggregationPlanNode: FastFilteredCount (COUNT only over an index-countable filter) and the
            # metadata plan (no filter; COUNT / MIN / MAX only) take the segment before the star-tree
            fns = {a.function for a in q.aggregations}
            if q.filter is None and "SUM" not in fns:
                f = None
            elif fns == {"COUNT"} and q.filter is not None and _index_countable(q, seg):
                f = None
        if f is None:
            r = O.execute(q, [seg])
            for key, row in zip(r.keys, r.aggs):
                fold(key, row)
            stats["num_docs_scanned"] += r.stats.num_docs_scanned
            stats["num_entries_scanned_in_filter"] += r.stats.num_entries_scanned_in_filter
            stats["num_entries_scanned_post_filter"] += r.stats.num_entries_scanned_post_filter
            stats["num_total_docs"] += r.stats.num_total_docs
            continue
        served += 1
        groups, (docs, ent, post, total) = execute(q, seg, st, *f)
        for key, row in groups.items():
            fold(key, row)
        stats["num_docs_scanned"] += docs
        stats["num_entries_scanned_in_filter"] += ent
        stats["num_entries_scanned_post_filter"] += post
        stats["num_total_docs"] += total
    if not q.group_by and not merged:
        merged[()] = [0 if a.function == "COUNT" else None for a in q.aggregations]
        order.append(())
    keys = order
    aggs = []
    for k in keys:
        row = []
        for j, a in enumerate(q.aggregations):
            v = merged[k][j]
            if v is None:  # an aggregation over no docs: the reference's default (SUM 0, MIN +inf, MAX -inf)
                v = {"COUNT": 0, "SUM": 0.0, "MIN": float("inf"), "MAX": float("-inf")}[a.function]
            row.append(v)
        aggs.append(row)
    return keys, aggs, stats, served


def _index_countable(q, seg) -> bool:
    """FastFilteredCountOperator's canOptimizeCount on the segment's own filter: sorted / inverted leaves and NOTs of
    them only (no scan, AND or OR)."""
    root = O._merge_same_column(O._plan_filter(q.filter, seg, {c: i for i, c in enumerate(seg.columns)}))

    def ok(n):
        if n.kind in ("all", "none"):
            return True
        if n.kind == "leaf":
            return getattr(n, "ikind", "") in ("sorted", "inverted")
        if n.kind == "not":
            return ok(n.children[0])
        return False
    return ok(root)
