// query.cpp -- host-side planning and execution of one query over pinned segments.
//
// Mirrors the reference's server plan for the filter -> aggregation / group-by shapes:
//   PredicateEvaluatorProvider.getPredicateEvaluator (core/operator/filter/predicate/PredicateEvaluatorProvider.java:45-96)
//     EQ    EqualsPredicateEvaluatorFactory.DictionaryBasedEqPredicateEvaluator    (:92-144)
//     NOT_EQ NotEqualsPredicateEvaluatorFactory (dictionary based)
//     IN    InPredicateEvaluatorFactory.DictionaryBasedInPredicateEvaluator          (:158-210)
//     NOT_IN NotInPredicateEvaluatorFactory.DictionaryBasedNotInPredicateEvaluator   (:158-210)
//     RANGE RangePredicateEvaluatorFactory.SortedDictionaryBasedRangePredicateEvaluator (:119-232)
//   FilterOperatorUtils.DefaultImplementation.getLeafFilterOperator (FilterOperatorUtils.java:73-125):
//     sorted column -> SortedIndexBasedFilterOperator (doc ranges); non-RANGE on an inverted column ->
//     InvertedIndexFilterOperator (doc bitmap); else ScanBasedFilterOperator (fused unpack + compare).
//   FilterPlanNode.constructPhysicalOperator (FilterPlanNode.java:200-318): AND drops match-all children
//     and is empty if any child is; OR drops empty children and matches all if any child does.
//   AggregationPlanNode (:95-150): no filter + only COUNT/MIN/MAX/DISTINCTCOUNTHLL -> answered from
//     dictionaries/metadata (NonScanBasedAggregationOperator).
//   GroupByPlanNode + DefaultGroupByExecutor + GroupByCombineOperator: one batched launch over every
//     segment, group keys over table-level global dictionaries so per-segment partial tables never need a
//     values-keyed merge (GroupByCombineOperator.java:169-178 keys by Object[] values; the global id is a
//     bijection with the value).
#include <algorithm>
#include <atomic>
#include <thread>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <set>
#include <unordered_map>

#include <functional>

#include "host_pool.h"
#include "ph_internal.h"

namespace ph {

namespace {

enum LeafKind { L_NONE, L_ALL, L_NODE };

// A physical filter node for one segment (before emission into the postfix program).
struct PNode {
  int kind = L_NODE;         // L_NONE / L_ALL / L_NODE
  int op = OP_RANGE;         // OP_* for leaves, OP_AND / OP_OR / OP_NOT for inner nodes
  int col = 0;               // slot
  uint32_t lo = 0, len = 0;
  std::vector<uint32_t> set;          // OP_SET bitset words
  std::vector<int32_t> ranges;        // OP_DOCRANGES pairs
  int bitmap_leaf = -1;               // OP_BITMAP: index into the query's bitmap list
  bool scan = false;
  bool exclusive = false;    // OP_NOT over OP_BITMAP built for an exclusive predicate (InvertedIndexFilterOperator's
                             // flipped bitmap: a BitmapDocIdSet, not a user NOT)
  bool range_index = false;  // a scan-evaluated RangeIndexBasedFilterOperator leaf: index-based for the statistics
  bool legacy_range = false;  // ... over a legacy version-1 index (its boundary ranges scanned: legacy_partial_entries)
  bool legacy_raw = false;    // ... whose index is over raw values: the predicate's inclusive raw bounds
  int64_t rlo_i = 0, rhi_i = 0;
  double rlo_d = 0, rhi_d = 0;
  bool range_pred = false;    // the leaf of a RANGE predicate (MergeRangeFilterOptimizer merges these under an AND)
  // AND whose children are index-based leaves (sorted, bitmap, range index, ORs / NOTs of them) followed by scan
  // leaves: the reference's AndDocIdSet applies the scans one after another to the index-based result
  // (ScanBasedDocIdIterator.applyAnd), so its filter entries are |D0| + |D0 n S1| + ... (counted on the device)
  int stats_nidx = 0, stats_nscan = 0;
  std::vector<PNode> kids;
};

struct BitmapLeaf {
  ph_segment* seg;
  Column* col;
  std::vector<int32_t> dict_ids;  // inverted-index leaf: the OR of these dictIds' bitmaps
  bool range = false;             // exact range-index leaf: dictIds [lo, hi] from the bit slices (k_range_slices)
  int64_t lo = 0, hi = -1;
  bool dead = false;              // merged into another range leaf (MergeRangeFilterOptimizer): never built
};

struct DictIdSet {
  // result of a dictionary-based predicate evaluator
  bool always_true = false, always_false = false;
  bool is_range = false;
  int64_t start = 0, end = 0;     // [start, end) when is_range
  std::vector<int32_t> ids;       // matching ids (sorted) when !is_range
  bool exclusive = false;         // NOT_EQ / NOT_IN: `ids` are the EXCLUDED ids
};

std::string lit(const char* s) { return s ? std::string(s) : std::string(); }

// Raw (no-dictionary) FLOAT / DOUBLE columns are dictionary-encoded at pin in Double.compare order (-0.0 before 0.0,
// NaN last), but the reference evaluates their predicates on the primitive values: EQ / IN `value == literal`
// (so 0 matches -0.0 and 0.0, NaN matches nothing), RANGE `value >= lo && value <= hi` with exclusive bounds moved
// by Math.nextUp / nextDown (NaN never matches), NOT_EQ / NOT_IN their complements (NaN included)
// (EqualsPredicateEvaluatorFactory / InPredicateEvaluatorFactory / RangePredicateEvaluatorFactory raw-value
// evaluators, e.g. RangePredicateEvaluatorFactory.java:482-522).  The matching dictIds are computed value by value.
DictIdSet evaluate_raw_real(const ph_predicate& p, const Column& c) {
  DictIdSet r;
  const Dictionary& d = c.dict;
  const int64_t card = d.size;
  const bool is_float = d.type == PH_FLOAT;
  auto parse = [&](const std::string& s) -> double {
    const char* b = s.c_str();
    char* e = nullptr;
    const double v = is_float ? (double)strtof(b, &e) : strtod(b, &e);
    if (e == b) fail(PH_ERR_BAD_QUERY, "not a number: " + s);
    return v;
  };
  std::vector<char> match((size_t)card, 0);
  bool exclusive = false;
  switch (p.type) {
    case PH_PRED_EQ:
    case PH_PRED_NOT_EQ:
    case PH_PRED_IN:
    case PH_PRED_NOT_IN: {
      if ((p.type == PH_PRED_EQ || p.type == PH_PRED_NOT_EQ) && (p.num_values != 1 || !p.values))
        fail(PH_ERR_BAD_QUERY, "EQ predicate needs one value");
      for (int i = 0; i < p.num_values; ++i) {
        const double x = parse(lit(p.values[i]));
        for (int64_t k = 0; k < card; ++k) match[k] |= d.reals[k] == x;
      }
      exclusive = p.type == PH_PRED_NOT_EQ || p.type == PH_PRED_NOT_IN;
      break;
    }
    case PH_PRED_RANGE: {
      const std::string lo = lit(p.lower), hi = lit(p.upper);
      double L = -INFINITY, U = INFINITY;
      if (p.lower && lo != "*") {
        L = parse(lo);
        if (!p.lower_inclusive) L = is_float ? (double)nextafterf((float)L, INFINITY) : nextafter(L, INFINITY);
      }
      if (p.upper && hi != "*") {
        U = parse(hi);
        if (!p.upper_inclusive) U = is_float ? (double)nextafterf((float)U, -INFINITY) : nextafter(U, -INFINITY);
      }
      for (int64_t k = 0; k < card; ++k) match[k] = d.reals[k] >= L && d.reals[k] <= U;
      break;
    }
    default:
      fail(PH_ERR_UNSUPPORTED, "predicate type " + std::to_string(p.type) + " is not on the GPU path");
  }
  std::vector<int32_t> ids;
  for (int64_t k = 0; k < card; ++k)
    if (match[k]) ids.push_back((int32_t)k);
  if (exclusive) {
    if (ids.empty()) { r.always_true = true; return r; }
    if ((int64_t)ids.size() == card) { r.always_false = true; return r; }
    r.exclusive = true;
    r.ids = std::move(ids);
    return r;
  }
  if (ids.empty()) { r.always_false = true; return r; }
  if ((int64_t)ids.size() == card) { r.always_true = true; return r; }
  if (ids.back() - ids.front() + 1 == (int32_t)ids.size()) {
    r.is_range = true;
    r.start = ids.front();
    r.end = ids.back() + 1;
  }
  r.ids = std::move(ids);
  return r;
}

DictIdSet evaluate_predicate(const ph_predicate& p, const Column& c) {
  if (c.is_raw && (c.dict.type == PH_FLOAT || c.dict.type == PH_DOUBLE)) return evaluate_raw_real(p, c);
  DictIdSet r;
  const Dictionary& d = c.dict;
  const int64_t card = d.size;
  switch (p.type) {
    case PH_PRED_EQ: {
      if (p.num_values != 1 || !p.values) fail(PH_ERR_BAD_QUERY, "EQ predicate needs one value");
      int64_t id = d.index_of(lit(p.values[0]));
      if (id < 0) { r.always_false = true; return r; }
      r.is_range = true;
      r.start = id;
      r.end = id + 1;
      r.always_true = card == 1;
      return r;
    }
    case PH_PRED_NOT_EQ: {
      if (p.num_values != 1 || !p.values) fail(PH_ERR_BAD_QUERY, "NOT_EQ predicate needs one value");
      int64_t id = d.index_of(lit(p.values[0]));
      if (id < 0) { r.always_true = true; return r; }
      if (card == 1) { r.always_false = true; return r; }
      r.exclusive = true;
      r.ids = {(int32_t)id};
      return r;
    }
    case PH_PRED_IN:
    case PH_PRED_NOT_IN: {
      std::vector<int32_t> ids;  // sorted, distinct
      ids.reserve((size_t)std::max(0, p.num_values));
      for (int i = 0; i < p.num_values; ++i) {
        int64_t id = d.index_of(lit(p.values[i]));
        if (id >= 0) ids.push_back((int32_t)id);
      }
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      if (p.type == PH_PRED_IN) {
        if (ids.empty()) { r.always_false = true; return r; }
        if ((int64_t)ids.size() == card) { r.always_true = true; return r; }
        r.ids = std::move(ids);
        if (r.ids.back() - r.ids.front() + 1 == (int32_t)r.ids.size()) {
          r.is_range = true;
          r.start = r.ids.front();
          r.end = r.ids.back() + 1;
        }
        return r;
      }
      if (ids.empty()) { r.always_true = true; return r; }
      if ((int64_t)ids.size() == card) { r.always_false = true; return r; }
      r.exclusive = true;
      r.ids = std::move(ids);
      return r;
    }
    case PH_PRED_RANGE: {
      const std::string lo = lit(p.lower), hi = lit(p.upper);
      int64_t start, end;
      // only "*" (RangePredicate.UNBOUNDED) or a missing bound is open: '' is a real (smallest) STRING literal
      if (!p.lower || lo == "*") {
        start = 0;
      } else {
        int64_t ii = d.insertion_index_of(lo);
        start = ii < 0 ? -(ii + 1) : (p.lower_inclusive ? ii : ii + 1);
      }
      if (!p.upper || hi == "*") {
        end = card;
      } else {
        int64_t ii = d.insertion_index_of(hi);
        end = ii < 0 ? -(ii + 1) : (p.upper_inclusive ? ii + 1 : ii);
      }
      if (end - start <= 0) { r.always_false = true; return r; }
      if (end - start == card) { r.always_true = true; return r; }
      r.is_range = true;
      r.start = start;
      r.end = end;
      return r;
    }
    default:
      fail(PH_ERR_UNSUPPORTED, "predicate type " + std::to_string(p.type) + " is not on the GPU path");
  }
}

// matching dictIds as sorted doc ranges of a sorted column (SortedIndexBasedFilterOperator)
std::vector<int32_t> sorted_doc_ranges(const Column& c, const DictIdSet& s) {
  std::vector<int32_t> ids;
  if (s.is_range) {
    for (int64_t i = s.start; i < s.end; ++i) ids.push_back((int32_t)i);
  } else if (s.exclusive) {
    size_t j = 0;
    for (int32_t i = 0; i < c.cardinality; ++i) {
      if (j < s.ids.size() && s.ids[j] == i) { ++j; continue; }
      ids.push_back(i);
    }
  } else {
    ids = s.ids;
  }
  std::vector<int32_t> out;
  for (int32_t id : ids) {
    int32_t a = c.sorted_ranges[2 * id], b = c.sorted_ranges[2 * id + 1];
    if (a > b) continue;
    if (!out.empty() && out.back() + 1 >= a) out.back() = std::max(out.back(), b);
    else { out.push_back(a); out.push_back(b); }
  }
  return out;
}

// A raw column's RANGE bounds as its raw-value evaluator holds them (RangePredicateEvaluatorFactory.java:70-92,
// :314-499): unbounded = the type's inclusive min / max (NEGATIVE / POSITIVE_INFINITY for reals), an exclusive bound
// moved by one (INT / LONG, int32 wrap-around for INT) or by Math.nextUp / nextDown (FLOAT / DOUBLE)
void raw_inclusive_bounds(const ph_predicate& p, int32_t type, int64_t* lo_i, int64_t* hi_i, double* lo_d, double* hi_d) {
  const std::string lo = lit(p.lower), hi = lit(p.upper);
  const bool lu = !p.lower || lo == "*", hu = !p.upper || hi == "*";
  const bool li = lu || p.lower_inclusive, hi_inc = hu || p.upper_inclusive;
  auto parse_i = [&](const std::string& v) {
    char* e = nullptr;
    const long long x = strtoll(v.c_str(), &e, 10);
    if (e == v.c_str() || *e) fail(PH_ERR_BAD_QUERY, "not an integer: " + v);
    return (int64_t)x;
  };
  auto parse_d = [&](const std::string& v) {
    char* e = nullptr;
    const double x = type == PH_FLOAT ? (double)strtof(v.c_str(), &e) : strtod(v.c_str(), &e);
    if (e == v.c_str()) fail(PH_ERR_BAD_QUERY, "not a number: " + v);
    return x;
  };
  if (type == PH_INT || type == PH_LONG) {
    const int64_t mn = type == PH_INT ? INT32_MIN : INT64_MIN, mx = type == PH_INT ? INT32_MAX : INT64_MAX;
    int64_t a = lu ? mn : parse_i(lo), b = hu ? mx : parse_i(hi);
    if (!li) a = type == PH_INT ? (int64_t)(int32_t)((uint32_t)a + 1u) : (int64_t)((uint64_t)a + 1u);
    if (!hi_inc) b = type == PH_INT ? (int64_t)(int32_t)((uint32_t)b - 1u) : (int64_t)((uint64_t)b - 1u);
    *lo_i = a;
    *hi_i = b;
  } else {
    double a = lu ? -INFINITY : parse_d(lo), b = hu ? INFINITY : parse_d(hi);
    if (!li) a = type == PH_FLOAT ? (double)nextafterf((float)a, INFINITY) : nextafter(a, INFINITY);
    if (!hi_inc) b = type == PH_FLOAT ? (double)nextafterf((float)b, -INFINITY) : nextafter(b, -INFINITY);
    *lo_d = a;
    *hi_d = b;
  }
}

struct Planner {
  const ph_query* q;
  std::map<std::string, int> slot;
  std::vector<BitmapLeaf> bitmaps;

  PNode leaf(ph_segment* seg, const ph_predicate& p) {
    if (!p.column) fail(PH_ERR_BAD_QUERY, "predicate without column");
    auto it = seg->columns.find(p.column);
    if (it == seg->columns.end()) fail(PH_ERR_BAD_QUERY, std::string("Column not found: ") + p.column);
    Column& c = *it->second;
    DictIdSet s = evaluate_predicate(p, c);
    PNode n;
    if (s.always_false) { n.kind = L_NONE; return n; }
    if (s.always_true) { n.kind = L_ALL; return n; }
    const int sl = slot.at(p.column);
    if (c.is_sorted) {
      n.op = OP_DOCRANGES;
      n.ranges = sorted_doc_ranges(c, s);
      if (n.ranges.empty()) { n.kind = L_NONE; return n; }
      if (n.ranges.size() == 2 && n.ranges[0] == 0 && n.ranges[1] >= seg->num_docs - 1) { n.kind = L_ALL; return n; }
      return n;
    }
    if (p.type != PH_PRED_RANGE && c.has_inverted()) {
      // InvertedIndexFilterOperator: OR of the matching bitmaps; exclusive predicates OR the excluded
      // bitmaps and flip (InvertedIndexFilterOperator.java:58-94)
      BitmapLeaf b{seg, &c, {}};
      if (s.is_range) for (int64_t i = s.start; i < s.end; ++i) b.dict_ids.push_back((int32_t)i);
      else b.dict_ids = s.ids;
      n.op = OP_BITMAP;
      n.bitmap_leaf = (int)bitmaps.size();
      bitmaps.push_back(std::move(b));
      if (s.exclusive) {
        PNode inv;
        inv.op = OP_NOT;
        inv.exclusive = true;
        inv.kids.push_back(std::move(n));
        return inv;
      }
      return n;
    }
    n.scan = true;
    n.col = sl;
    // RangeIndexBasedFilterOperator (FilterOperatorUtils.java:97-120; canEvaluate :56-61): RANGE on a column with an
    // exact range index, or EQ on one without an inverted index.  Same doc set as a scan of the dictIds, which is
    // how the kernels evaluate it; it scans no entries (BitmapDocIdSet)
    n.range_index = c.has_range_index && (p.type == PH_PRED_RANGE || (p.type == PH_PRED_EQ && !c.has_inverted()));
    if (n.range_index && c.range_slices && !s.exclusive && (s.is_range || s.ids.size() == 1)) {
      // BitSlicedRangeIndexReader.getMatchingDocIds(min, max) / (value) (:123-171): the dictId interval's doc
      // bitmap from the index's slices; a bitmap-based leaf like an inverted one (RangeIndexBasedFilterOperator
      // :78-92), priority 200 in the AND order
      BitmapLeaf b{seg, &c, {}};
      b.range = true;
      b.lo = s.is_range ? s.start : s.ids[0];
      b.hi = s.is_range ? s.end - 1 : s.ids[0];
      n.scan = false;
      n.col = -1;
      n.op = OP_BITMAP;
      n.range_pred = p.type == PH_PRED_RANGE;
      n.bitmap_leaf = (int)bitmaps.size();
      bitmaps.push_back(std::move(b));
      return n;
    }
    // a legacy version-1 range index evaluates RANGE only (RangeIndexBasedFilterOperator.canEvaluate :56-61): a
    // BitmapDocIdSet of the exact docs (scanned from the dictIds here) whose entries are the scan of its boundary
    // ranges (evaluateLegacyRangeFilter :82-107), added per segment by legacy_partial_entries
    if (c.has_inexact_range_index && p.type == PH_PRED_RANGE && (c.legacy_range || c.legacy_raw)) {
      n.range_index = true;
      n.legacy_range = true;
      if (c.legacy_raw) {
        n.legacy_raw = true;
        raw_inclusive_bounds(p, c.data_type, &n.rlo_i, &n.rhi_i, &n.rlo_d, &n.rhi_d);
      }
    }
    if (s.is_range) {
      n.op = OP_RANGE;
      n.lo = (uint32_t)s.start;
      n.len = (uint32_t)(s.end - s.start);
      return n;
    }
    n.op = OP_SET;
    n.set.assign(((size_t)c.cardinality + 31) / 32, s.exclusive ? 0xffffffffu : 0u);
    for (int32_t id : s.ids) {
      if (s.exclusive) n.set[id >> 5] &= ~(1u << (id & 31));
      else n.set[id >> 5] |= 1u << (id & 31);
    }
    return n;
  }

  PNode build(ph_segment* seg, int node_index, int depth) {
    if (depth > 64) fail(PH_ERR_UNSUPPORTED, "filter tree too deep");
    if (node_index < 0 || node_index >= q->num_filter_nodes) fail(PH_ERR_INVALID_ARGUMENT, "bad filter node index");
    const ph_filter_node& f = q->filter_nodes[node_index];
    switch (f.type) {
      case PH_FILTER_PREDICATE:
        if (f.predicate < 0 || f.predicate >= q->num_predicates) fail(PH_ERR_INVALID_ARGUMENT, "bad predicate index");
        return leaf(seg, q->predicates[f.predicate]);
      case PH_FILTER_AND: {
        PNode n;
        n.op = OP_AND;
        for (int i = 0; i < f.num_children; ++i) {
          PNode k = build(seg, f.children[i], depth + 1);
          if (k.kind == L_NONE) { PNode e; e.kind = L_NONE; return e; }
          if (k.kind == L_ALL) continue;
          n.kids.push_back(std::move(k));
        }
        if (n.kids.empty()) { PNode a; a.kind = L_ALL; return a; }
        if (n.kids.size() == 1) return std::move(n.kids[0]);
        return n;
      }
      case PH_FILTER_OR: {
        PNode n;
        n.op = OP_OR;
        for (int i = 0; i < f.num_children; ++i) {
          PNode k = build(seg, f.children[i], depth + 1);
          if (k.kind == L_ALL) { PNode a; a.kind = L_ALL; return a; }
          if (k.kind == L_NONE) continue;
          n.kids.push_back(std::move(k));
        }
        if (n.kids.empty()) { PNode e; e.kind = L_NONE; return e; }
        if (n.kids.size() == 1) return std::move(n.kids[0]);
        return n;
      }
      case PH_FILTER_NOT: {
        if (f.num_children != 1) fail(PH_ERR_INVALID_ARGUMENT, "NOT needs exactly one child");
        PNode k = build(seg, f.children[0], depth + 1);
        if (k.kind == L_ALL) { PNode e; e.kind = L_NONE; return e; }
        if (k.kind == L_NONE) { PNode a; a.kind = L_ALL; return a; }
        PNode n;
        n.op = OP_NOT;
        n.kids.push_back(std::move(k));
        return n;
      }
      default:
        fail(PH_ERR_INVALID_ARGUMENT, "bad filter node type");
    }
  }
};

// [first, end) docs a segment's filter can match: sorted doc ranges bound it, an AND intersects, an OR takes the hull
std::pair<int64_t, int64_t> doc_span(const PNode& n, int64_t docs) {
  if (n.kind == L_NONE) return {0, 0};
  if (n.kind == L_ALL) return {0, docs};
  if (n.op == OP_DOCRANGES && !n.ranges.empty())
    return {n.ranges.front(), std::min<int64_t>(docs, (int64_t)n.ranges.back() + 1)};
  if (n.op == OP_AND) {
    std::pair<int64_t, int64_t> r{0, docs};
    for (auto& k : n.kids) {
      auto x = doc_span(k, docs);
      r = {std::max(r.first, x.first), std::min(r.second, x.second)};
    }
    if (r.second < r.first) r = {0, 0};
    return r;
  }
  if (n.op == OP_OR) {
    std::pair<int64_t, int64_t> r{docs, 0};
    for (auto& k : n.kids) {
      auto x = doc_span(k, docs);
      if (x.second > x.first) r = {std::min(r.first, x.first), std::max(r.second, x.second)};
    }
    if (r.second < r.first) r = {0, 0};
    return r;
  }
  return {0, docs};
}

// Same-column scan leaves under one AND / OR combine into one leaf (intersection / union of their dictId sets:
// `d_year >= 1992 AND d_year <= 1997` -> one range, `c_city = 'A' OR c_city = 'B'` -> one set), the dictId-space
// form of what the reference evaluates as separate ScanBasedFilterOperators; results are unchanged.  A set whose
// ids are contiguous becomes a range.
std::vector<uint32_t> leaf_bits(const PNode& k, int64_t card) {
  if (k.op == OP_SET) {
    std::vector<uint32_t> b = k.set;
    b.resize((size_t)(card + 31) / 32, 0u);
    return b;
  }
  std::vector<uint32_t> b((size_t)(card + 31) / 32, 0u);
  for (int64_t i = k.lo; i < (int64_t)k.lo + k.len && i < card; ++i) b[i >> 5] |= 1u << (i & 31);
  return b;
}

void leaf_from_bits(PNode& n, const std::vector<uint32_t>& b, int64_t card) {
  int64_t first = -1, last = -1, count = 0;
  for (int64_t i = 0; i < card; ++i)
    if ((b[i >> 5] >> (i & 31)) & 1u) {
      if (first < 0) first = i;
      last = i;
      ++count;
    }
  if (count == 0) {
    n = PNode{};
    n.kind = L_NONE;
    return;
  }
  if (count == card) {
    n = PNode{};
    n.kind = L_ALL;
    return;
  }
  if (count == last - first + 1) {
    n.op = OP_RANGE;
    n.lo = (uint32_t)first;
    n.len = (uint32_t)count;
    n.set.clear();
  } else {
    n.op = OP_SET;
    n.set = b;
  }
}

template <class CardOf>
void merge_same_column_leaves(PNode& n, const CardOf& card_of, std::vector<BitmapLeaf>* bms = nullptr) {
  if (n.kind != L_NODE) return;
  for (auto& k : n.kids) merge_same_column_leaves(k, card_of, bms);
  if (n.op != OP_AND && n.op != OP_OR) return;
  if (n.stats_nscan) return;  // its scan children stay separate: each is one applyAnd step of the statistic
  const bool is_and = n.op == OP_AND;
  std::map<int, size_t> first_of;  // column slot -> index of its first scan leaf
  std::map<const Column*, size_t> first_range;  // column -> index of its first slice-evaluated RANGE leaf
  std::vector<PNode> kids;
  for (auto& k : n.kids) {
    // RANGE leaves of one column under an AND evaluated from the range index's slices: one leaf over the
    // intersected dictId interval (MergeRangeFilterOptimizer.java:50-100 merges the predicates before planning, so
    // the reference builds one RangeIndexBasedFilterOperator, or an EmptyFilterOperator for an empty interval)
    if (is_and && bms && k.kind == L_NODE && k.op == OP_BITMAP && k.range_pred && (*bms)[k.bitmap_leaf].range) {
      BitmapLeaf& b = (*bms)[k.bitmap_leaf];
      auto it = first_range.find(b.col);
      if (it != first_range.end()) {
        PNode& a = kids[it->second];
        if (a.kind == L_NONE) {
          b.dead = true;
          continue;
        }
        BitmapLeaf& ab = (*bms)[a.bitmap_leaf];
        ab.lo = std::max(ab.lo, b.lo);
        ab.hi = std::min(ab.hi, b.hi);
        b.dead = true;
        if (ab.hi < ab.lo) {
          ab.dead = true;
          a = PNode{};
          a.kind = L_NONE;
        }
        continue;
      }
      first_range[b.col] = kids.size();
    }
    // a legacy range-index leaf merges only with another under an AND (MergeRangeFilterOptimizer: one RANGE,
    // planned once); the other scans merge as before, never with it
    const bool legacy = k.kind == L_NODE && k.legacy_range;
    if (k.kind == L_NODE && k.scan && (k.op == OP_RANGE || k.op == OP_SET) && (!legacy || is_and)) {
      const int key = legacy ? -2 - k.col : k.col;
      auto it = first_of.find(key);
      if (it != first_of.end()) {
        PNode& a = kids[it->second];
        const int64_t card = card_of(k.col);
        std::vector<uint32_t> x = leaf_bits(a, card), y = leaf_bits(k, card);
        for (size_t w = 0; w < x.size(); ++w) x[w] = is_and ? (x[w] & y[w]) : (x[w] | y[w]);
        const PNode ka = a;
        leaf_from_bits(a, x, card);
        if (legacy && ka.legacy_raw && a.kind == L_NODE) {  // the merged RANGE's raw bounds (MergeRangeFilterOptimizer)
          a.range_index = a.legacy_range = a.legacy_raw = true;
          a.rlo_i = std::max(ka.rlo_i, k.rlo_i);
          a.rhi_i = std::min(ka.rhi_i, k.rhi_i);
          a.rlo_d = std::max(ka.rlo_d, k.rlo_d);
          a.rhi_d = std::min(ka.rhi_d, k.rhi_d);
        }
        continue;
      }
      first_of[key] = kids.size();
    }
    kids.push_back(std::move(k));
  }
  std::vector<PNode> out;
  for (auto& k : kids) {
    if (k.kind == (is_and ? L_NONE : L_ALL)) {  // AND with an empty child / OR with an all child
      n = PNode{};
      n.kind = is_and ? L_NONE : L_ALL;
      return;
    }
    if (k.kind == (is_and ? L_ALL : L_NONE)) continue;
    out.push_back(std::move(k));
  }
  if (out.empty()) {
    n = PNode{};
    n.kind = is_and ? L_ALL : L_NONE;
    return;
  }
  if (out.size() == 1) {
    PNode only = std::move(out[0]);
    n = std::move(only);
    return;
  }
  n.kids = std::move(out);
}

// scan leaves whose entries are numDocs each (a lone scan, scans under an OR, a pure-scan AND -- the latter an
// approximation of AndDocIdIterator's advance-driven count); the scans of an applyAnd AND are counted on the device
int count_scan_leaves(const PNode& n) {
  if (n.kind != L_NODE) return 0;
  int s = (n.scan && !n.range_index) ? 1 : 0;
  for (size_t i = 0; i < n.kids.size(); ++i)
    if (!(n.stats_nscan && (int)i >= n.stats_nidx)) s += count_scan_leaves(n.kids[i]);
  return s;
}

// a child whose docIdSet iterator is Sorted- or BitmapBased (AndDocIdSet.java:80-100)
bool index_based(const PNode& k) {
  if (k.kind != L_NODE) return false;
  if (k.op == OP_DOCRANGES || k.op == OP_BITMAP) return true;
  if (k.scan) return k.range_index;
  if (k.op == OP_NOT) return k.exclusive;  // exclusive inverted-index leaf (a user NOT is a NotDocIdSet)
  if (k.op == OP_OR) {
    for (auto& c : k.kids)
      if (!index_based(c)) return false;
    return !k.kids.empty();
  }
  return false;
}

// flag the ANDs of index-based children + scan leaves (and order their children as the reference does: index-based
// first, scans after them in their original order -- every SV scan has SCAN_PRIORITY, FilterOperatorUtils.java:197-241)
void mark_apply_and(PNode& n) {
  if (n.kind != L_NODE) return;
  if (n.op == OP_AND) {
    std::vector<PNode> idx, scans;
    bool ok = true;
    for (auto& k : n.kids) {
      if (index_based(k)) idx.push_back(k);
      else if (k.scan && k.kids.empty()) scans.push_back(k);
      else ok = false;
    }
    if (ok && !idx.empty() && !scans.empty() && scans.size() <= 16) {
      n.stats_nidx = (int)idx.size();
      n.stats_nscan = (int)scans.size();
      n.kids.clear();
      for (auto& k : idx) n.kids.push_back(std::move(k));
      for (auto& k : scans) n.kids.push_back(std::move(k));
      return;
    }
  }
  for (auto& k : n.kids) mark_apply_and(k);
}

// How a segment's numEntriesScannedInFilter is computed (the reference counts the docs its scan iterators examine,
// which depends on how its iterator tree drives them: filter_sim.cpp):
//  ST_DEVICE  -- every scan is either drained by next() (a lone scan, scans under an OR / a NOT of a leaf: numDocs
//                each) or applied by an AndDocIdSet to its merged index-based children (applyAnd: |D0| + |D0 n S1| +
//                ..., counted per doc by the flagged AND of the device program / FK_CONJ / k_group_sparse);
//  ST_SCANAND -- an AND of SV scans only: AndDocIdIterator leap-frogs their advance() (k_scan_and_entries);
//  ST_SIM     -- anything else: the host runs the iterator tree over the leaves' doc bitmaps (k_filter_bitmaps).
enum StatKind { ST_DEVICE = 0, ST_SCANAND = 1, ST_SIM = 2 };

bool plain_scan(const PNode& k) { return k.kind == L_NODE && k.scan && !k.range_index && k.kids.empty(); }
// a leaf of the reference's operator tree: a predicate leaf, or an exclusive inverted leaf (its flipped bitmap)
bool stat_leaf(const PNode& k) { return k.kind == L_NODE && (k.kids.empty() || (k.op == OP_NOT && k.exclusive)); }

int stat_kind(const PNode& r) {
  if (r.kind != L_NODE || stat_leaf(r)) return ST_DEVICE;
  auto leafish = [](const PNode& k) { return stat_leaf(k) || (k.op == OP_NOT && stat_leaf(k.kids[0])); };
  if (r.op == OP_NOT) return leafish(r) ? ST_DEVICE : ST_SIM;
  if (r.op == OP_OR) {
    for (auto& k : r.kids)
      if (!leafish(k)) return ST_SIM;
    return ST_DEVICE;
  }
  int nidx = 0, nscan = 0;
  for (auto& k : r.kids) {
    if (index_based(k)) ++nidx;
    else if (plain_scan(k)) ++nscan;
    else return ST_SIM;
  }
  if (nidx > 0) return nscan <= 16 ? ST_DEVICE : ST_SIM;  // mark_apply_and flags up to 16 scans
  return nscan <= kMaxFbProgs ? ST_SCANAND : ST_SIM;
}

// the statistic's tree of a segment for the host simulation: leaves collected in order (one doc bitmap each)
SimNode to_sim(const PNode& n, std::vector<PNode>& leaves, std::vector<int32_t>& kinds) {
  SimNode x;
  if (stat_leaf(n)) {
    x.op = SIM_LEAF;
    x.leaf = (int32_t)leaves.size();
    leaves.push_back(n);
    // FilterOperatorUtils priorities (:197-241): SortedIndexBasedFilterOperator 0, RangeIndexBasedFilterOperator 200,
    // ScanBasedFilterOperator 500; InvertedIndexFilterOperator is none of the listed classes (10000)
    if (n.op == OP_DOCRANGES) { kinds.push_back(SIM_SORTED); x.priority = 0; }
    else if (n.range_index) { kinds.push_back(SIM_BITMAP); x.priority = 200; }  // scan- or slice-evaluated
    else if (n.scan) { kinds.push_back(SIM_SCAN); x.priority = 500; }
    else { kinds.push_back(SIM_BITMAP); x.priority = 10000; }
    return x;
  }
  x.op = n.op == OP_AND ? SIM_AND : (n.op == OP_OR ? SIM_OR : SIM_NOT);
  x.priority = n.op == OP_AND ? 300 : 400;
  for (auto& k : n.kids) x.kids.push_back(to_sim(k, leaves, kinds));
  return x;
}

void clear_apply_and(PNode& n) {
  n.stats_nidx = n.stats_nscan = 0;
  for (auto& k : n.kids) clear_apply_and(k);
}

// k_group_sparse's filter shape: one inverted-index leaf, or an AND of 1..kMaxConj of them and <= kMaxConj plain
// scan leaves (dictId range / set; the applyAnd order of mark_apply_and: index-based kids first)
struct SparseShape {
  bool ok = false;
  std::vector<std::vector<int>> groups;  // AND of ORs of bitmap leaves
  std::vector<const PNode*> scans;       // scan leaves, in order
};
SparseShape sparse_shape(const PNode& r) {
  SparseShape sh;
  auto is_bitmap = [](const PNode& k) { return k.kind == L_NODE && k.op == OP_BITMAP; };
  auto bitmap_or = [&](const PNode& k) {
    if (k.kind != L_NODE || k.op != OP_OR || k.kids.empty()) return false;
    for (auto& c : k.kids)
      if (!is_bitmap(c)) return false;
    return true;
  };
  auto is_scan = [](const PNode& k) {
    return k.kind == L_NODE && k.scan && !k.range_index && k.kids.empty() && (k.op == OP_RANGE || k.op == OP_SET);
  };
  auto add_index = [&](const PNode& k) {
    if (is_bitmap(k)) {
      sh.groups.push_back({k.bitmap_leaf});
      return true;
    }
    if (!bitmap_or(k)) return false;
    sh.groups.emplace_back();
    for (auto& c : k.kids) sh.groups.back().push_back(c.bitmap_leaf);
    return true;
  };
  if (r.kind == L_NODE && r.op == OP_AND) {
    for (auto& k : r.kids) {
      if (add_index(k)) continue;
      if (!is_scan(k)) return sh;
      sh.scans.push_back(&k);
    }
  } else if (!add_index(r)) {
    return sh;
  }
  size_t nbm = 0;
  for (auto& g : sh.groups) nbm += g.size();
  // no bitmaps: an AND of >= 2 scan leaves, evaluated register-direct by the sparse kernels (conj_reg.h)
  sh.ok = nbm <= (size_t)kSparseBitmaps && (int)sh.scans.size() <= kMaxConj &&
          (!sh.groups.empty() || sh.scans.size() >= 2);
  return sh;
}

// host-side storage of a segment's program before device upload
struct SegProgram {
  std::vector<FilterInsn> insns;
  std::vector<std::pair<size_t, std::vector<uint32_t>>> payloads;  // insn index -> words (set / ranges)
  std::vector<std::pair<size_t, int>> bitmap_refs;                 // insn index -> bitmap leaf
  int depth = 0, max_depth = 0;
  bool apply_and = false;  // the program counts applyAnd filter entries (FilterInsn OP_AND with len > 0)
};

void emit(const PNode& n, SegProgram& p) {
  FilterInsn in{};
  if (n.op == OP_AND || n.op == OP_OR || n.op == OP_NOT) {
    for (auto& k : n.kids) emit(k, p);
    in.op = n.op;
    in.col = (int32_t)n.kids.size();
    if (n.op == OP_AND && n.stats_nscan) {  // applyAnd statistic: index-based children, then scan children
      in.lo = (uint32_t)n.stats_nidx;
      in.len = (uint32_t)n.stats_nscan;
      p.apply_and = true;
    }
    if (n.op != OP_NOT) p.depth -= (int)n.kids.size() - 1;
    p.insns.push_back(in);
    return;
  }
  in.op = n.op;
  in.col = n.col;
  in.lo = n.lo;
  in.len = n.len;
  if (n.op == OP_SET) p.payloads.push_back({p.insns.size(), n.set});
  if (n.op == OP_DOCRANGES) {
    in.lo = (uint32_t)(n.ranges.size() / 2);
    std::vector<uint32_t> w(n.ranges.begin(), n.ranges.end());
    p.payloads.push_back({p.insns.size(), w});
  }
  if (n.op == OP_BITMAP) p.bitmap_refs.push_back({p.insns.size(), n.bitmap_leaf});
  p.insns.push_back(in);
  p.depth++;
  p.max_depth = std::max(p.max_depth, p.depth);
}

// docs of the dictIds' bitmaps: a single-value column's bitmaps are disjoint, so the OR's cardinality is the sum
// (InvertedIndexFilterOperator.getNumMatchingDocs :101-127)
// RangeIndexReaderImpl.findRangeId over dictIds (:236-243)
int64_t legacy_range_id(const Column& c, int64_t v) {
  for (size_t i = 0; i < c.legacy_starts.size(); ++i)
    if (v < c.legacy_starts[i]) return (int64_t)i - 1;
  return v <= c.legacy_last_end ? (int64_t)c.legacy_starts.size() - 1 : (int64_t)c.legacy_starts.size();
}
// RangeIndexReaderImpl.findRangeId(double / float) (:257-273): reals compared in the index's type (a float widened to
// double keeps its order)
int64_t legacy_range_id_real(const Column& c, double v) {
  for (size_t i = 0; i < c.legacy_rstarts.size(); ++i)
    if (v < c.legacy_rstarts[i]) return (int64_t)i - 1;
  return v <= c.legacy_rlast_end ? (int64_t)c.legacy_rstarts.size() - 1 : (int64_t)c.legacy_rstarts.size();
}

// the legacy range-index leaves' boundary-range scans of one segment's (merged) tree: getPartialMatchesInRange
// (RangeIndexReaderImpl.java:300-308) of the leaf's inclusive dictId bounds, counted by ScanBasedDocIdIterator.applyAnd
// (SVScanDocIdIterator.java:115-140); every leaf's getTrues runs, whatever the tree above it
template <class ColOf>
int64_t legacy_partial_entries(const PNode& n, const ColOf& col_of) {
  if (n.kind != L_NODE) return 0;
  int64_t e = 0;
  for (auto& k : n.kids) e += legacy_partial_entries(k, col_of);
  if (!n.legacy_range || !n.kids.empty()) return e;
  const Column& c = col_of(n.col);
  if (n.legacy_raw) {  // over raw values: the predicate's inclusive raw bounds
    const int64_t R = (int64_t)c.legacy_cards.size();
    const bool real = c.data_type == PH_FLOAT || c.data_type == PH_DOUBLE;
    const int64_t a = real ? legacy_range_id_real(c, n.rlo_d) : legacy_range_id(c, n.rlo_i);
    const int64_t b = real ? legacy_range_id_real(c, n.rhi_d) : legacy_range_id(c, n.rhi_i);
    if (a >= 0 && a < R) e += c.legacy_cards[a];
    if (b >= 0 && b < R && b != a) e += c.legacy_cards[b];
    return e;
  }
  int64_t lo = -1, hi = -1;
  if (n.op == OP_RANGE) {
    lo = n.lo;
    hi = (int64_t)n.lo + n.len - 1;
  } else {
    for (int64_t i = 0; i < (int64_t)n.set.size() * 32; ++i)
      if ((n.set[i >> 5] >> (i & 31)) & 1u) {
        if (lo < 0) lo = i;
        hi = i;
      }
    if (lo < 0) return e;
  }
  const int64_t R = (int64_t)c.legacy_starts.size();
  const int64_t a = legacy_range_id(c, lo), b = legacy_range_id(c, hi);
  if (a >= 0 && a < R) e += c.legacy_cards[a];
  if (b >= 0 && b < R && b != a) e += c.legacy_cards[b];
  return e;
}

int64_t bitmap_docs(const Column& c, const std::vector<int32_t>& ids) {
  int64_t n = 0;
  for (int32_t id : ids) n += c.id_docs[id];
  return n;
}

// a bitmap leaf's docs for the plan's cost estimates: exact for an inverted leaf; a range-index leaf's count is not
// known before its bitmap is built, so uniform dictIds are assumed
double leaf_docs_estimate(const BitmapLeaf& b) {
  if (!b.range) return (double)bitmap_docs(*b.col, b.dict_ids);
  return (double)b.seg->num_docs * (double)(b.hi - b.lo + 1) / (double)std::max<int32_t>(1, b.col->cardinality);
}

// FastFilteredCountOperator's getNumMatchingDocs from the index alone (AggregationPlanNode.java:183-188): a sorted doc
// range, an inverted-index bitmap (disjoint per dictId in a single-value column) or their NOT; -1 when the filter
// needs a scan (AND / OR / scan leaves, range-slice leaves counted from their bitmap)
int64_t index_count(const PNode& n, const std::vector<BitmapLeaf>& bms, int64_t docs) {
  if (n.kind == L_ALL) return docs;
  if (n.kind == L_NONE) return 0;
  if (n.op == OP_DOCRANGES) {
    int64_t c = 0;
    for (size_t r = 0; r + 1 < n.ranges.size(); r += 2) c += (int64_t)n.ranges[r + 1] - n.ranges[r] + 1;
    return c;
  }
  if (n.op == OP_BITMAP) {
    const BitmapLeaf& b = bms[(size_t)n.bitmap_leaf];
    if (b.range) return -1;
    return bitmap_docs(*b.col, b.dict_ids);
  }
  if (n.op == OP_NOT && n.kids.size() == 1) {
    const int64_t c = index_count(n.kids[0], bms, docs);
    return c < 0 ? -1 : docs - c;
  }
  return -1;
}

// a star-tree view's filter (StarTreeFilterOperator.getFilterOperator, StarTreeFilterOperator.java:157-199): the
// traversal's documents (a BitmapBasedFilterOperator: index-based, first in the AND) AND each remaining composite --
// one predicate's leaf, or the OR of its predicates' leaves -- over the view's dimension columns
PNode star_root(Planner& pl, ph_segment* seg, const StarSegPlan& sp) {
  PNode none;
  none.kind = L_NONE;
  if (sp.empty || sp.ranges.empty()) return none;
  PNode docs;
  docs.op = OP_DOCRANGES;
  docs.ranges = sp.ranges;
  PNode a;
  a.op = OP_AND;
  a.kids.push_back(std::move(docs));
  for (auto& comp : sp.composites) {
    PNode k;
    if (comp.size() == 1) {
      k = pl.leaf(seg, pl.q->predicates[comp[0]]);
    } else {
      k.op = OP_OR;
      bool all = false;
      for (int32_t pi : comp) {
        PNode x = pl.leaf(seg, pl.q->predicates[pi]);
        if (x.kind == L_ALL) all = true;
        if (x.kind == L_NODE) k.kids.push_back(std::move(x));
      }
      if (all) k.kind = L_ALL;
      else if (k.kids.empty()) k.kind = L_NONE;
      else if (k.kids.size() == 1) k = std::move(k.kids[0]);
    }
    if (k.kind == L_NONE) return none;
    if (k.kind == L_ALL) continue;
    a.kids.push_back(std::move(k));
  }
  if (a.kids.size() == 1) return std::move(a.kids[0]);
  return a;
}

}  // namespace

namespace {

// ------------------------------------------------------------------ global dictionaries
std::shared_ptr<GlobalDict> build_union(Context* ctx, const std::string& col, const std::vector<ph_segment*>& segs) {
  Dictionary u;
  const Column* first = nullptr;
  for (auto* s : segs) {
    auto it = s->columns.find(col);
    if (it == s->columns.end()) fail(PH_ERR_BAD_QUERY, "Column not found: " + col);
    if (!first) first = it->second.get();
    else if (it->second->data_type != first->data_type) fail(PH_ERR_BAD_QUERY, "column " + col + " has mixed types");
  }
  if (!first) fail(PH_ERR_INVALID_ARGUMENT, "no segments");
  u.type = first->data_type;
  if (u.type == PH_STRING) {
    std::vector<std::string> all;
    for (auto* s : segs) {
      auto& d = s->columns.at(col)->dict;
      all.insert(all.end(), d.strings.begin(), d.strings.end());
    }
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    u.strings = std::move(all);
    for (auto& x : u.strings) u.max_string_len = std::max<int32_t>(u.max_string_len, (int32_t)x.size());
    u.size = (int64_t)u.strings.size();
  } else if (u.type == PH_INT || u.type == PH_LONG) {
    std::vector<int64_t> all;
    for (auto* s : segs) {
      auto& d = s->columns.at(col)->dict;
      all.insert(all.end(), d.ints.begin(), d.ints.end());
    }
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    u.ints = std::move(all);
    u.size = (int64_t)u.ints.size();
  } else {
    std::vector<double> all;
    for (auto* s : segs) {
      auto& d = s->columns.at(col)->dict;
      all.insert(all.end(), d.reals.begin(), d.reals.end());
    }
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    u.reals = std::move(all);
    u.size = (int64_t)u.reals.size();
  }
  auto g = std::make_shared<GlobalDict>();
  g->dict = std::move(u);
  g->id = next_object_id();
  return g;
}

// dictId -> global id; nullptr when identity
const int32_t* segment_remap(Context* ctx, const ph_segment& s, const Column& c, GlobalDict& g) {
  std::lock_guard<std::mutex> lk(g.mu);
  auto it = g.remaps.find(s.id);
  if (it != g.remaps.end()) return it->second ? it->second->as<int32_t>() : nullptr;
  std::vector<int32_t> map(c.cardinality);
  bool identity = c.cardinality == g.dict.size;
  int64_t j = 0;
  for (int32_t i = 0; i < c.cardinality; ++i) {
    while (j < g.dict.size && g.dict.compare(j, c.dict, i) < 0) ++j;
    if (j >= g.dict.size || g.dict.compare(j, c.dict, i) != 0)
      fail(PH_ERR_INVALID_ARGUMENT, "table dictionary of column " + c.name + " does not contain a segment value");
    map[i] = (int32_t)j;
    identity &= (j == i);
  }
  std::shared_ptr<DeviceBuffer> buf;
  if (!identity) {
    buf = std::make_shared<DeviceBuffer>();
    buf->alloc(sizeof(int32_t) * map.size(), ctx->device);
    copy_h2d_sync(buf->ptr, map.data(), sizeof(int32_t) * map.size());
  }
  g.remaps[s.id] = buf;
  return buf ? buf->as<int32_t>() : nullptr;
}

// table-level dictionary values on the device (group-key decoding in the compaction kernel)
const void* global_dict_device_values(Context* ctx, GlobalDict& g) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (g.dict.type == PH_STRING) return nullptr;
  if (!g.d_values) {
    auto b = std::make_unique<DeviceBuffer>();
    const int64_t n = std::max<int64_t>(1, g.dict.size);
    b->alloc(8 * n, ctx->device);
    const void* src = (g.dict.type == PH_INT || g.dict.type == PH_LONG) ? (const void*)g.dict.ints.data()
                                                                        : (const void*)g.dict.reals.data();
    copy_h2d_sync(b->ptr, src, 8 * g.dict.size);
    g.d_values = std::move(b);
  }
  return g.d_values->ptr;
}

const uint32_t* segment_hll_table(Context* ctx, Column& c, int log2m, hipStream_t st) {
  {
    std::lock_guard<std::mutex> lk(c.cache_mu);
    auto it = c.hll_tables.find(log2m);
    if (it != c.hll_tables.end()) return it->second.buf->as<uint32_t>();
  }
  // not built at pin (ph_column_desc.hll_log2m): the first query that needs it does
  std::lock_guard<std::mutex> lk(c.cache_mu);
  build_hll_table(ctx, c, log2m, st);
  PH_HIP_CHECK(hipStreamSynchronize(st));
  return c.hll_tables.at(log2m).buf->as<uint32_t>();
}

void put_key_value(const Dictionary& d, int64_t id, uint8_t* dst, int32_t entry) {
  switch (d.type) {
    case PH_INT: { int32_t v = (int32_t)d.ints[id]; memcpy(dst, &v, 4); break; }
    case PH_LONG: memcpy(dst, &d.ints[id], 8); break;
    case PH_FLOAT: { float v = (float)d.reals[id]; memcpy(dst, &v, 4); break; }
    case PH_DOUBLE: memcpy(dst, &d.reals[id], 8); break;
    default: {
      memset(dst, 0, entry);
      memcpy(dst, d.strings[id].data(), std::min<size_t>(entry, d.strings[id].size()));
    }
  }
}

int32_t key_entry_size(const Dictionary& d) {
  switch (d.type) {
    case PH_INT: case PH_FLOAT: return 4;
    case PH_LONG: case PH_DOUBLE: return 8;
    default: return std::max(1, d.max_string_len);
  }
}

double value_as_double(const Dictionary& d, int64_t i) {
  return (d.type == PH_INT || d.type == PH_LONG) ? (double)d.ints[i] : d.reals[i];
}

}  // namespace

// scratch device allocation living for one query
// Per-query device buffers drawn from the context's scratch pool and returned to it when the query ends
// (every query synchronises its stream before returning, so nothing is in flight by then).
struct QueryScratch {
  std::vector<std::unique_ptr<DeviceBuffer>> bufs;
  Context* ctx;
  hipStream_t st, sb;  // the call's streams: drained before the buffers go back to the pool
  QueryScratch(Context* c, hipStream_t s1, hipStream_t s2) : ctx(c), st(s1), sb(s2) {}
  ~QueryScratch() {
    (void)hipStreamSynchronize(st);
    (void)hipStreamSynchronize(sb);
    for (auto& b : bufs) ctx->scratch_release(std::move(b));
  }
  template <class T>
  T* alloc(size_t count) {
    auto b = ctx->scratch_acquire(std::max<size_t>(16, sizeof(T) * count));
    T* p = b->as<T>();
    bufs.push_back(std::move(b));
    return p;
  }
};

namespace {

int bits_for_range(uint64_t range) {
  int b = 0;
  while (b < 64 && (range >> b) != 0) ++b;
  return b;
}

// Frame-of-reference value stream of an INT/LONG column (VK_PACKED), built once per pinned column.
// the frame-of-reference value stream of an INT / LONG column (VK_PACKED), built at pin (build_value_stream)
bool ensure_value_stream(Context*, ph_segment*, Column& c, hipStream_t) { return c.d_vpacked != nullptr; }

}  // namespace

void fill_tile_pieces(DevSegment& d, int nstage, const int32_t* stage_soff, int tile_words) {
  int np = 0;
  for (int s = 0; s < nstage; ++s) {
    const int bits = d.streams[s].bits;
    if (!bits) continue;
    const int n = stage_loads(tile_words, bits);
    for (int i = 0; i < n; ++i) {
      if (np >= kMaxPieces) fail(PH_ERR_UNSUPPORTED, "tile pieces exceed the prefetch pool");
      DevPiece& pc = d.pieces[np++];
      pc.fwd = reinterpret_cast<const uint8_t*>(d.streams[s].fwd) + 1024 * i;
      pc.stride = 8 * bits;
      pc.off = 1024 * i;
      pc.lds = stage_soff[s] + 16 + 1024 * i;
    }
  }
  d.npieces = np;
}

// the sorted value union of a column over segments (any devices'): a table-level dictionary for one query
std::shared_ptr<GlobalDict> union_dictionary(const std::string& col, const std::vector<ph_segment*>& segs) {
  return build_union(nullptr, col, segs);
}

std::vector<char> predicate_dict_ids(const ph_predicate& p, const Column& c, bool* always_true, bool* always_false) {
  const DictIdSet s = evaluate_predicate(p, c);
  *always_true = s.always_true;
  *always_false = s.always_false;
  std::vector<char> m((size_t)std::max(0, c.cardinality), 0);
  if (s.always_false) return m;
  if (s.always_true) {
    std::fill(m.begin(), m.end(), 1);
    return m;
  }
  if (s.is_range) {
    for (int64_t i = s.start; i < s.end && i < (int64_t)m.size(); ++i) m[(size_t)i] = 1;
    return m;
  }
  if (s.exclusive) std::fill(m.begin(), m.end(), 1);
  for (int32_t id : s.ids)
    if (id >= 0 && id < (int32_t)m.size()) m[(size_t)id] = s.exclusive ? 0 : 1;
  return m;
}

bool filter_index_countable(const ph_query* q, ph_segment* seg) {
  if (q->filter_root < 0) return true;
  Planner pl;
  pl.q = q;
  std::vector<std::string> names;
  for (int i = 0; i < q->num_predicates; ++i)
    if (q->predicates[i].column && !pl.slot.count(q->predicates[i].column)) {
      pl.slot[q->predicates[i].column] = (int)names.size();
      names.push_back(q->predicates[i].column);
    }
  PNode root = pl.build(seg, q->filter_root, 0);
  merge_same_column_leaves(root, [&](int slot) { return (int64_t)seg->columns.at(names[(size_t)slot])->cardinality; },
                           &pl.bitmaps);
  return index_count(root, pl.bitmaps, seg->num_docs) >= 0;
}

ph_result* query_execute_impl(Context* ctx, const ph_query* q, ph_segment* const* segs_in, int32_t nseg,
                              const DenseArgs* dn) {
  const int dop = dn ? dn->op : 0;
  const bool fin = dop == DENSE_FINALIZE;
  // ph_filter_execute: a COUNT(*) (no group-by) whose MODE_COUNT scan also writes every segment's doc bitmap
  const FilterDocset* fds = (dn && !dop) ? dn->docset : nullptr;
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  const bool host_times = getenv("PH_HOST_TIMES") != nullptr;  // per-phase host clock (tuning)
  auto stamp = [&](const char* what) {
    if (host_times)
      fprintf(stderr, "[ph host] %-12s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(clock::now() - t0).count());
  };
  if (!q) fail(PH_ERR_INVALID_ARGUMENT, "null query");
  if (nseg < 0 || (nseg > 0 && !segs_in)) fail(PH_ERR_INVALID_ARGUMENT, "bad segment list");
  if (q->num_aggregations > kMaxAggs) fail(PH_ERR_UNSUPPORTED, "too many aggregations");
  if (fds && (q->num_group_by != 0 || q->num_aggregations != 1 || q->aggregations[0].type != PH_AGG_COUNT ||
              q->filter_root < 0))
    fail(PH_ERR_INVALID_ARGUMENT, "a filter call is a filtered COUNT(*)");
  if (q->num_group_by > kMaxGroupCols) fail(PH_ERR_UNSUPPORTED, "too many group-by columns");
  // segments a star-tree serves (GroupByPlanNode.java:77-99, AggregationPlanNode.java:122-141): their views, merged
  // with the rest (startree.cpp)
  const std::map<const ph_segment*, StarSegPlan>* star = dn ? dn->star : nullptr;
  if (!star && !fds && !q->skip_star_tree && nseg > 0)
    if (ph_result* r = star_tree_execute(ctx, q, segs_in, nseg, dop)) return r;
  PH_HIP_CHECK(hipSetDevice(ctx->device));
  LaneGuard lane(ctx);  // this call's streams, events and staging (concurrent calls use their own)
  const hipStream_t st = lane.stream();
  std::vector<ph_segment*> segs(segs_in, segs_in + nseg);
  for (auto* s : segs)
    if (!s || s->ctx != ctx) fail(PH_ERR_INVALID_ARGUMENT, "segment is null or pinned on another context");

  // BaseOperator.nextBlock's interruption check (BaseOperator.java:39) and the combine's end time
  // (GroupByCombineOperator.java:225-234), at the points where a call can stop without work in flight
  const bool interruptible = q->interrupt != nullptr || q->end_time_ms > 0;
  auto check_interrupt = [&]() {
    if (q->interrupt && *q->interrupt) fail(PH_ERR_CANCELLED, "query interrupted");
    if (q->end_time_ms > 0) {
      const int64_t now = std::chrono::duration_cast<std::chrono::milliseconds>(
                              std::chrono::system_clock::now().time_since_epoch()).count();
      if (now > q->end_time_ms) fail(PH_ERR_CANCELLED, "query timed out (end time passed)");
    }
  };
  check_interrupt();
  auto res = std::make_unique<ph_result>();
  ph_exec_stats& stats = res->stats;
  stats.num_segments_processed = nseg;
  for (auto* s : segs) stats.num_total_docs += s->num_docs;

  // ---- columns / slots
  Planner pl;
  pl.q = q;
  std::vector<std::string> slot_names;
  auto add_slot = [&](const std::string& c) {
    if (!pl.slot.count(c)) {
      pl.slot[c] = (int)slot_names.size();
      slot_names.push_back(c);
    }
  };
  std::vector<std::string> group_cols;
  for (int g = 0; g < q->num_group_by; ++g) {
    if (!q->group_by || !q->group_by[g]) fail(PH_ERR_INVALID_ARGUMENT, "null group-by column");
    group_cols.push_back(q->group_by[g]);
    add_slot(q->group_by[g]);
  }
  // aggregation -> (value column, op) / HLL register set
  const int nagg = q->num_aggregations;
  int log2m = 0;
  // value terms: a column, or a 2-operand expression `val_cols[j] <op> val_cols2[j]`
  std::vector<std::string> val_cols, val_cols2, hll_cols;
  std::vector<int> val_ops, val_exprs;
  std::vector<int> agg_val(nagg, -1), agg_hll(nagg, -1);
  std::set<std::string> projected(group_cols.begin(), group_cols.end());
  for (int k = 0; k < nagg; ++k) {
    const ph_aggregation& a = q->aggregations[k];
    if (a.type < PH_AGG_COUNT || a.type > PH_AGG_DISTINCTCOUNTHLL) fail(PH_ERR_UNSUPPORTED, "aggregation type");
    res->agg_types.push_back(a.type);
    const int lm = a.type == PH_AGG_DISTINCTCOUNTHLL ? (a.log2m > 0 ? a.log2m : 8) : 0;
    res->agg_log2m.push_back(lm);
    if (a.type == PH_AGG_COUNT) continue;
    if (!a.column) fail(PH_ERR_BAD_QUERY, "aggregation needs a column");
    add_slot(a.column);
    projected.insert(a.column);
    if (a.type == PH_AGG_DISTINCTCOUNTHLL) {
      if (lm < 4 || lm > 16) fail(PH_ERR_UNSUPPORTED, "log2m out of range");
      if (log2m && lm != log2m) fail(PH_ERR_UNSUPPORTED, "DISTINCTCOUNTHLL with different log2m in one query");
      log2m = lm;
      auto it = std::find(hll_cols.begin(), hll_cols.end(), std::string(a.column));
      if (it == hll_cols.end()) {
        if ((int)hll_cols.size() >= kMaxHll) fail(PH_ERR_UNSUPPORTED, "too many DISTINCTCOUNTHLL columns");
        hll_cols.push_back(a.column);
        agg_hll[k] = (int)hll_cols.size() - 1;
      } else {
        agg_hll[k] = (int)(it - hll_cols.begin());
      }
      continue;
    }
    const int eop = a.expr_op;
    if (eop < PH_EXPR_NONE || eop > PH_EXPR_ADD) fail(PH_ERR_UNSUPPORTED, "expression operator");
    const std::string col2 = eop ? lit(a.column2) : std::string();
    if (eop) {
      if (!a.column2) fail(PH_ERR_BAD_QUERY, "expression needs a second operand");
      add_slot(col2);
      projected.insert(col2);
    }
    int j = -1;
    for (size_t t = 0; t < val_cols.size(); ++t)
      if (val_cols[t] == a.column && val_exprs[t] == eop && val_cols2[t] == col2) j = (int)t;
    if (j < 0) {
      if ((int)val_cols.size() >= kMaxVals) fail(PH_ERR_UNSUPPORTED, "too many aggregated columns");
      val_cols.push_back(a.column);
      val_cols2.push_back(col2);
      val_exprs.push_back(eop);
      val_ops.push_back(0);
      j = (int)val_cols.size() - 1;
    }
    agg_val[k] = j;
    val_ops[j] |= a.type == PH_AGG_SUM ? 1 : (a.type == PH_AGG_MIN ? 2 : 4);
  }
  const int nvals = (int)val_cols.size(), num_hll = (int)hll_cols.size();
  if (q->filter_root >= 0)
    for (int i = 0; i < q->num_predicates; ++i) {
      if (!q->predicates[i].column) fail(PH_ERR_BAD_QUERY, "predicate without column");
      add_slot(q->predicates[i].column);
    }
  if ((int)slot_names.size() > kMaxCols) fail(PH_ERR_UNSUPPORTED, "too many columns in one query");
  std::vector<int> val_is_int(nvals, 1);
  for (auto* s : segs)
    for (auto& c : slot_names) {
      auto it = s->columns.find(c);
      if (it == s->columns.end()) fail(PH_ERR_BAD_QUERY, "Column not found: " + c + " in segment " + s->name);
    }
  // |value| bound of term j over the queried segments (integer terms only; 0 when unknown)
  std::vector<double> term_amax(nvals, 0.0);
  for (int j = 0; j < nvals; ++j) {
    int is_int = 1;
    double amax[2] = {0.0, 0.0};
    for (int o = 0; o < (val_exprs[j] ? 2 : 1); ++o) {
      const std::string& cn = o ? val_cols2[j] : val_cols[j];
      int col_int = -1;
      for (size_t i = 0; i < segs.size(); ++i) {
        const Column& c = *segs[i]->columns.at(cn);
        const int dt = c.data_type;
        if (dt == PH_STRING) fail(PH_ERR_UNSUPPORTED, "numeric aggregation on STRING column " + cn);
        const int ci = dt == PH_INT || dt == PH_LONG;
        if (col_int < 0) col_int = ci;
        else if (col_int != ci)
          fail(PH_ERR_UNSUPPORTED, "aggregation column with mixed integer/real types across segments");
        if (ci && c.cardinality > 0) {
          amax[o] = std::max(amax[o], std::fabs((double)c.dict.ints.front()));
          amax[o] = std::max(amax[o], std::fabs((double)c.dict.ints.back()));
        }
      }
      if (col_int < 0) {  // no queried segment holds it: the schema type (ph_table_set_column_type)
        std::lock_guard<std::mutex> dlk(ctx->mu);
        auto ct = ctx->column_types.find(cn);
        if (ct != ctx->column_types.end()) {
          if (ct->second == PH_STRING) fail(PH_ERR_UNSUPPORTED, "numeric aggregation on STRING column " + cn);
          col_int = ct->second == PH_INT || ct->second == PH_LONG;
        } else if (dop) {
          fail(PH_ERR_INVALID_ARGUMENT, "dense call without segments needs ph_table_set_column_type for " + cn);
        }
      }
      is_int &= col_int != 0;
    }
    double bound = amax[0];
    if (val_exprs[j] == PH_EXPR_MULT) bound = amax[0] * amax[1];
    else if (val_exprs[j]) bound = amax[0] + amax[1];
    // an integer expression is exact in int64 only while it cannot overflow; else double arithmetic, as the
    // reference computes it
    if (val_exprs[j] && bound >= 4.0e18) is_int = 0;
    val_is_int[j] = is_int;
    term_amax[j] = is_int ? bound : 0.0;
  }
  const int m = log2m ? (1 << log2m) : 0;

  // ---- aggregation-only, no filter, metadata-answerable (NonScanBasedAggregationOperator)
  bool non_scan = q->filter_root < 0 && q->num_group_by == 0 && nagg > 0;
  for (int k = 0; k < nagg && non_scan; ++k) non_scan = q->aggregations[k].type != PH_AGG_SUM;
  if (dop || star) non_scan = false;  // dense partials always come from the scan; a view's filter is its traversal
  res->num_groups = 1;
  auto init_row_results = [&](int64_t rows) {
    res->aggs.resize(nagg);
    for (int k = 0; k < nagg; ++k) {
      const int t = q->aggregations[k].type;
      size_t w = t == PH_AGG_DISTINCTCOUNTHLL ? (size_t)(1 << res->agg_log2m[k]) : 8;
      res->aggs[k].assign(w * rows, 0);
    }
  };
  if (non_scan) {
    init_row_results(1);
    for (int k = 0; k < nagg; ++k) {
      const ph_aggregation& a = q->aggregations[k];
      if (a.type == PH_AGG_COUNT) {
        int64_t v = stats.num_total_docs;
        memcpy(res->aggs[k].data(), &v, 8);
      } else if (a.type == PH_AGG_MIN || a.type == PH_AGG_MAX) {
        double v = a.type == PH_AGG_MIN ? INFINITY : -INFINITY;
        for (auto* s : segs) {
          Column& c = *s->columns.at(a.column);
          if (c.cardinality == 0 || s->num_docs == 0) continue;
          double x = value_as_double(c.dict, a.type == PH_AGG_MIN ? 0 : c.cardinality - 1);
          v = a.type == PH_AGG_MIN ? std::min(v, x) : std::max(v, x);
        }
        memcpy(res->aggs[k].data(), &v, 8);
      } else {  // DISTINCTCOUNTHLL from the dictionaries
        uint8_t* regs = res->aggs[k].data();
        const int lm = res->agg_log2m[k];
        for (auto* s : segs) {
          Column& c = *s->columns.at(a.column);
          if (s->num_docs == 0) continue;
          const uint32_t* dt = segment_hll_table(ctx, c, lm, st);
          std::vector<uint32_t> h(c.cardinality);
          PH_HIP_CHECK(hipMemcpy(h.data(), dt, sizeof(uint32_t) * h.size(), hipMemcpyDeviceToHost));
          for (uint32_t e : h) regs[e >> 8] = std::max<uint8_t>(regs[e >> 8], (uint8_t)(e & 0xff));
        }
      }
    }
    stats.num_docs_scanned = stats.num_total_docs;
    stats.num_segments_matched = nseg;
    stats.plan_mode = -1;
    stats.host_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    return res.release();
  }

  stamp("pre-plan");
  // ---- per-segment filter plans
  QueryScratch scratch(ctx, st, lane.lane->stream_b);
  if (fds && fds->total_words > 0) PH_HIP_CHECK(hipMemsetAsync(fds->words, 0, 8 * (size_t)fds->total_words, st));
  std::vector<SegProgram> progs(nseg);
  std::vector<PNode> roots(nseg);
  std::vector<char> seg_live(nseg, 1);
  // segments whose filter statistic runs a pass of its own (ST_SCANAND / ST_SIM): the reference's tree over the
  // leaves, the leaves themselves (one doc bitmap each) and their iterator kinds
  struct StatSeg {
    int qi, kind;
    SimNode root;
    std::vector<PNode> leaves;
    std::vector<int32_t> leaf_kinds;
    int32_t dseg = -1;
    std::vector<size_t> jobs;  // its FbJobs (<= kMaxFbProgs leaves each) for the leaves k_leaf_bitmaps does not take
    // an AND of scans whose leaves the sparse kernels' register-direct front end evaluates anyway (conj_reg.h): it
    // writes their doc bitmaps here (leaf-major, ceil(docs / 64) words each), so the walk reads no forward index
    unsigned long long* fused = nullptr;
  };
  // a leaf k_leaf_bitmaps computes from the forward index: a dictId range or a small dictId set of a scan leaf
  auto fast_leaf = [&](const PNode& n) {
    return n.kind == L_NODE && n.scan && n.kids.empty() &&
           (n.op == OP_RANGE || (n.op == OP_SET && n.set.size() <= (size_t)kLeafSetWords));
  };
  std::vector<StatSeg> stat_segs;
  pl.bitmaps.reserve(pl.bitmaps.size() + (size_t)nseg * 2);
  double tacc[8] = {};
  auto tnow = [&]() { return host_times ? clock::now() : clock::time_point{}; };
  auto tadd = [&](int k, clock::time_point a) {
    if (host_times) tacc[k] += std::chrono::duration<double, std::milli>(clock::now() - a).count();
  };
  for (int i = 0; i < nseg && dop != DENSE_LAYOUT && !fin; ++i) {
    auto ta = tnow();
    PNode root;
    root.kind = L_ALL;
    auto sv = star ? star->find(segs[i]) : decltype(star->end()){};
    if (star && sv != star->end()) root = star_root(pl, segs[i], sv->second);
    else if (q->filter_root >= 0) root = pl.build(segs[i], q->filter_root, 0);
    tadd(0, ta);
    ta = tnow();
    // same-column scan predicates merge first, as the reference's query optimizer merges them before planning
    // (MergeEqInFilterOptimizer: `d_year = 1997 OR d_year = 1998` -> one IN; MergeRangeFilterOptimizer: ranges of
    // one column under an AND), so the statistics below see the reference's operator tree
    merge_same_column_leaves(
        root, [&](int slot) { return (int64_t)segs[i]->columns.at(slot_names[slot])->cardinality; }, &pl.bitmaps);
    if (segs[i]->num_docs > 0)
      stats.num_entries_scanned_in_filter += legacy_partial_entries(
          root, [&](int slot) -> const Column& { return *segs[i]->columns.at(slot_names[slot]); });
    tadd(1, ta);
    ta = tnow();
    const int sk = stat_kind(root);
    if (sk != ST_DEVICE && segs[i]->num_docs > 0) {
      StatSeg ss;
      ss.qi = i;
      ss.kind = sk;
      ss.root = to_sim(root, ss.leaves, ss.leaf_kinds);
      stat_segs.push_back(std::move(ss));
    }
    mark_apply_and(root);
    if (sk != ST_DEVICE) clear_apply_and(root);  // the pass counts this segment, not the device program
    else stats.num_entries_scanned_in_filter += (int64_t)segs[i]->num_docs * count_scan_leaves(root);
    if (root.kind == L_NONE || segs[i]->num_docs == 0) seg_live[i] = 0;
    roots[i] = std::move(root);
    tadd(2, ta);
  }
  if (host_times) fprintf(stderr, "[ph host]   plans: build %.3f merge+legacy %.3f stat+mark %.3f ms\n", tacc[0], tacc[1], tacc[2]);

  // ---- FastFilteredCountOperator (AggregationPlanNode.java:183-188): COUNT only, and every segment's filter
  // answers getNumMatchingDocs from its index -- a sorted doc range, an inverted-index bitmap (disjoint per
  // dictId in a single-value column) or their NOT -- so no doc is scanned
  bool fast_count = q->num_group_by == 0 && nagg > 0 && q->filter_root >= 0 && !dop && !fds;
  for (int k = 0; k < nagg && fast_count; ++k) fast_count = q->aggregations[k].type == PH_AGG_COUNT;
  if (fast_count) {
    auto count_of = [&](const PNode& n, int64_t docs) { return index_count(n, pl.bitmaps, docs); };
    int64_t total = 0;
    for (int i = 0; i < nseg && fast_count; ++i) {
      if (!seg_live[i]) continue;
      const int64_t c = count_of(roots[i], segs[i]->num_docs);
      if (c < 0) fast_count = false;
      total += c;
    }
    if (fast_count) {
      init_row_results(1);
      for (int k = 0; k < nagg; ++k) memcpy(res->aggs[k].data(), &total, 8);
      stats.num_docs_scanned = total;
      for (int i = 0; i < nseg; ++i) stats.num_segments_matched += seg_live[i] ? 1 : 0;
      stats.plan_mode = -2;
      res->mode = -2;
      stats.host_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
      return res.release();
    }
  }

  // ---- inverted-index leaves -> device doc bitmaps
  // (container lists from the directories cached at pin; one upload for all leaves)
  std::vector<uint32_t*> bitmap_dev(pl.bitmaps.size(), nullptr);
  auto build_bitmaps = [&]() {
    if (pl.bitmaps.empty() || dop == DENSE_LAYOUT || fin) return;
    // all leaves' bitmaps in one block, each padded to whole 64-doc words + one
    const size_t nl = pl.bitmaps.size();
    std::vector<size_t> woff(nl + 1, 0);
    bool chunked = !ctx->has(OPT_ROARING_ATOMIC);  // option roaring_atomic: the device-atomic build (tests)
    for (size_t i = 0; i < nl; ++i) {
      woff[i + 1] = woff[i] + (((size_t)pl.bitmaps[i].seg->num_docs + 63) / 64 + 1) * 2;
      const Column& col = *pl.bitmaps[i].col;
      for (int32_t id : pl.bitmaps[i].dict_ids)
        chunked = chunked && col.dir_begin[id + 1] - col.dir_begin[id] <= kRoaringChunkMaxContainers;
    }
    uint32_t* block = scratch.alloc<uint32_t>(std::max<size_t>(2, woff.back()));
    for (size_t i = 0; i < nl; ++i) bitmap_dev[i] = block + woff[i];
    // range-index leaves: k_range_slices writes every word of theirs (after the atomic build's memset, below)
    auto build_range_leaves = [&]() {
      std::vector<RangeSliceLeaf> rl;
      int max_chunks = 0;
      for (size_t i = 0; i < nl; ++i) {
        const BitmapLeaf& b = pl.bitmaps[i];
        if (!b.range || b.dead) continue;
        const Column& col = *b.col;
        const int32_t pw = (int32_t)(woff[i + 1] - woff[i]);
        RangeSliceLeaf L{};
        L.payload = col.d_range.as<uint8_t>();
        L.dir = col.d_range_dir.as<int32_t>();
        L.bitmap = bitmap_dev[i];
        L.num_docs = b.seg->num_docs;
        L.padded_words = pw;
        L.nkeys = col.range_nkeys;
        L.nslices = col.range_nslices;
        L.hi = (uint64_t)b.hi;  // <= cardinality - 1 < 2^nslices (checked at pin)
        L.use_lo = b.lo > 0;
        L.lo_m1 = b.lo > 0 ? (uint64_t)(b.lo - 1) : 0;
        rl.push_back(L);
        max_chunks = std::max(max_chunks, (pw + 2047) / 2048);
      }
      if (rl.empty()) return;
      const size_t bytes = sizeof(RangeSliceLeaf) * rl.size();
      uint8_t* dev = scratch.alloc<uint8_t>(bytes);
      uint8_t* stage = static_cast<uint8_t*>(lane.lane->host_staging(bytes, 3));
      memcpy(stage, rl.data(), bytes);
      PH_HIP_CHECK(hipMemcpyAsync(dev, stage, bytes, hipMemcpyHostToDevice, st));
      launch_range_slices(reinterpret_cast<RangeSliceLeaf*>(dev), (int)rl.size(), max_chunks, st);
    };
    if (chunked) {
      // k_roaring_chunk: one workgroup per (65536-doc chunk, leaf) builds the chunk in LDS and stores every word
      std::vector<RoaringLeaf> lv(nl);
      std::vector<RoaringRange> rg;
      int max_chunks = 0;
      for (size_t i = 0; i < nl; ++i) {
        if (pl.bitmaps[i].range) continue;
        const Column& col = *pl.bitmaps[i].col;
        const int32_t first = (int32_t)rg.size();
        for (int32_t id : pl.bitmaps[i].dict_ids) {
          const int64_t f = col.dir_begin[id], n = col.dir_begin[id + 1] - f;
          if (n > 0) rg.push_back(RoaringRange{(int32_t)f, (int32_t)n});
        }
        const int32_t pw = (int32_t)(woff[i + 1] - woff[i]);
        lv[i] = RoaringLeaf{col.d_inverted.as<uint8_t>(), col.d_dir.as<RoaringContainer>(), bitmap_dev[i],
                            pl.bitmaps[i].seg->num_docs, pw, first, (int32_t)rg.size() - first};
        max_chunks = std::max(max_chunks, (pw + 2047) / 2048);
      }
      lv.erase(std::remove_if(lv.begin(), lv.end(), [](const RoaringLeaf& l) { return l.bitmap == nullptr; }),
               lv.end());
      if (!lv.empty()) {
        const size_t b1 = sizeof(RoaringLeaf) * lv.size(), b2 = sizeof(RoaringRange) * std::max<size_t>(1, rg.size());
        uint8_t* dev = scratch.alloc<uint8_t>(b1 + b2);
        // staging slot 1: nothing else in this call writes it, so the build overlaps the rest of the host setup
        uint8_t* stage = static_cast<uint8_t*>(lane.lane->host_staging(b1 + b2, 1));
        memcpy(stage, lv.data(), b1);
        if (!rg.empty()) memcpy(stage + b1, rg.data(), sizeof(RoaringRange) * rg.size());
        PH_HIP_CHECK(hipMemcpyAsync(dev, stage, b1 + b2, hipMemcpyHostToDevice, st));
        launch_roaring_chunk(reinterpret_cast<RoaringLeaf*>(dev), (int)lv.size(), max_chunks,
                             reinterpret_cast<RoaringRange*>(dev + b1), st);
      }
      build_range_leaves();
      return;
    }
    // device-atomic build: a zeroed block, every container of every leaf OR-ed in by ONE launch
    std::vector<RoaringWork> cs;  // items of (leaf, dictId, <= 16 containers); the containers stay in the directories
    std::vector<RoaringTarget> tg(nl);
    for (size_t i = 0; i < nl; ++i) {
      const Column& col = *pl.bitmaps[i].col;
      if (pl.bitmaps[i].range) continue;  // its target stays unused
      for (int32_t id : pl.bitmaps[i].dict_ids) {
        const int64_t f = col.dir_begin[id], n = col.dir_begin[id + 1] - f;
        for (int64_t k = 0; k < n; k += kRoaringWorkContainers)  // 4 containers per wave keeps the grid wide
          cs.push_back(RoaringWork{col.d_dir.as<RoaringContainer>(), (int32_t)i, (int32_t)(f + k),
                                   (int32_t)std::min<int64_t>(kRoaringWorkContainers, n - k), 0});
      }
      tg[i] = RoaringTarget{col.d_inverted.as<uint8_t>(), bitmap_dev[i], pl.bitmaps[i].seg->num_docs, 0};
    }
    PH_HIP_CHECK(hipMemsetAsync(block, 0, 4 * std::max<size_t>(2, woff.back()), st));
    if (!cs.empty()) {
      const size_t b1 = sizeof(RoaringWork) * cs.size(), b2 = sizeof(RoaringTarget) * tg.size();
      uint8_t* dev = scratch.alloc<uint8_t>(b1 + b2);
      uint8_t* stage = static_cast<uint8_t*>(lane.lane->host_staging(b1 + b2, 1));
      memcpy(stage, cs.data(), b1);
      memcpy(stage + b1, tg.data(), b2);
      PH_HIP_CHECK(hipMemcpyAsync(dev, stage, b1 + b2, hipMemcpyHostToDevice, st));
      launch_roaring_or(reinterpret_cast<RoaringWork*>(dev), (int)cs.size(), reinterpret_cast<RoaringTarget*>(dev + b1),
                        st);
    }
    build_range_leaves();  // after the memset: k_range_slices writes every word of its leaves
  };
  stamp("plan");
  // Aggregation-only queries whose every segment is filtered by ONE inverted leaf (EQ / IN) may run k_agg_sparse
  // straight from the leaf's roaring containers (KParams::agg_cont, decided with the sparse plan below): the dictIds
  // of a single-value column have disjoint doc sets, so the leaf's docs are the disjoint union of its ids'
  // containers and no doc bitmap is needed.  The bitmaps are built only if that plan is not taken
  bool cont_defer = q->num_group_by == 0 && !pl.bitmaps.empty() && dop != DENSE_LAYOUT && !fin;
  if (ctx->has(OPT_AGG_CONT)) cont_defer = cont_defer && ctx->opt(OPT_AGG_CONT) != 0;
  {
    int live = 0;
    for (int i = 0; i < nseg && cont_defer; ++i) {
      if (!seg_live[i]) continue;
      ++live;
      const PNode& r = roots[i];
      cont_defer = r.kind == L_NODE && r.op == OP_BITMAP && !r.exclusive && r.bitmap_leaf >= 0 &&
                   !pl.bitmaps[r.bitmap_leaf].range;
    }
    cont_defer = cont_defer && live == (int)pl.bitmaps.size();  // no other bitmap leaf anywhere
  }
  // Group-bys whose every segment's filter is a sparse_shape AND with bitmap leaves (SSB Q2-Q4 on inverted
  // dimensions) may run k_group_sparse with each chunk's leaf bitmaps built in LDS from the containers
  // (KParams::group_cont, decided with the sparse plan below): their doc bitmaps too are built only if not taken.
  // Opt-in (PH_GROUP_CONT=1): r5 measured the inverted SSB flight at 15.2 ms of kernels against 10.7 with
  // k_roaring_chunk's bitmaps -- the per-chunk build (container search, byte-wise payload reads, LDS atomics, two
  // barriers) serialises in front of every chunk's gathers, where the separate build runs fully parallel
  bool gs_defer = ctx->has(OPT_GROUP_CONT) && ctx->opt(OPT_GROUP_CONT) != 0 && q->num_group_by > 0 && !pl.bitmaps.empty() && dop != DENSE_LAYOUT && !fin;
  {
    size_t leaves = 0;
    for (int i = 0; i < nseg && gs_defer; ++i) {
      if (!seg_live[i]) continue;
      const SparseShape sh = sparse_shape(roots[i]);
      gs_defer = sh.ok && !sh.groups.empty();
      for (auto& g : sh.groups) leaves += g.size();
    }
    gs_defer = gs_defer && leaves == pl.bitmaps.size();  // no bitmap leaf outside the sparse ANDs
    for (auto& b : pl.bitmaps) gs_defer = gs_defer && !b.range;
  }
  // the bitmap build's device time is part of the query's device_ms (its own event pair: host setup follows it)
  bool bm_timed = false;
  if (!pl.bitmaps.empty() && dop != DENSE_LAYOUT && !fin && !cont_defer && !gs_defer) {
    PH_HIP_CHECK(hipEventRecord(lane.lane->ev_bm0, st));
    build_bitmaps();
    PH_HIP_CHECK(hipEventRecord(lane.lane->ev_bm1, st));
    bm_timed = true;
  }
  stamp("bitmaps");

  // ---- group-by key space over table-level dictionaries
  std::vector<std::shared_ptr<GlobalDict>> gdicts;
  int64_t num_groups = 1;
  for (auto& g : group_cols) {
    std::shared_ptr<GlobalDict> gd;
    std::lock_guard<std::mutex> dlk(ctx->mu);  // table dictionaries / union cache
    auto it = ctx->table_dicts.find(g);
    if (dn && dn->dicts) {
      gd = (*dn->dicts).at(gdicts.size());
    } else if (it != ctx->table_dicts.end()) {
      gd = it->second;
    } else {
      std::string key = g + "#";
      for (auto* s : segs) key += std::to_string(s->id) + ",";
      auto ct = ctx->union_cache.find(key);
      if (ct != ctx->union_cache.end()) {
        gd = ct->second;
      } else {
        gd = build_union(ctx, g, segs);
        // bounded FIFO of unions; an evicted union's per-segment remaps go with it (segment_remap purges them)
        while (ctx->union_cache.size() >= kUnionCacheEntries) {
          ctx->union_cache.erase(ctx->union_order.front());
          ctx->union_order.pop_front();
        }
        ctx->union_cache[key] = gd;
        ctx->union_order.push_back(key);
      }
    }
    gdicts.push_back(gd);
    const int64_t sz = std::max<int64_t>(1, gd->dict.size);
    // mixed-radix keys stay below 2^62 (int64 and never the hash table's empty marker)
    if (num_groups > (int64_t(1) << 62) / sz) fail(PH_ERR_UNSUPPORTED, "group key space too large");
    num_groups *= sz;
  }
  // numGroupsLimit (per segment): a segment whose product of group-by cardinalities reaches the limit may hit it;
  // such segments get a first-seen pass before the scan (DictionaryBasedGroupKeyGenerator keeps the first
  // `limit` keys in doc order and drops the rest, IntGroupIdMap.getGroupId :992-1017; GroupByOperator.java:111
  // reports numGroups >= limit)
  const int64_t group_limit = q->num_groups_limit > 0 ? q->num_groups_limit : 100000;
  std::vector<char> seg_limit(nseg, 0);
  bool any_limit = false;
  if (q->num_group_by > 0 && dop != DENSE_LAYOUT && !fin) {
    for (int i = 0; i < nseg; ++i) {
      if (!seg_live[i]) continue;
      // a segment holds at most min(product of cardinalities, docs) distinct keys
      int64_t pp = 1;
      for (auto& g : group_cols) {
        const int64_t c = std::max<int64_t>(1, segs[i]->columns.at(g)->cardinality);
        pp = pp > (int64_t(1) << 40) / c ? int64_t(1) << 40 : pp * c;
      }
      if (std::min<int64_t>(pp, segs[i]->num_docs) >= group_limit) seg_limit[i] = any_limit = true;
    }
  }
  const int64_t G = num_groups;
  if (dop) {
    // partial tables of different GPUs line up only over table-level dictionaries
    std::lock_guard<std::mutex> dlk(ctx->mu);
    for (auto& g : group_cols)
      if (!ctx->table_dicts.count(g) && !dn->dicts)
        fail(PH_ERR_INVALID_ARGUMENT, "dense partials need ph_table_set_dictionary for group-by column " + g);
    if (fin && (dn->g0 < 0 || dn->g1 < dn->g0 || dn->g1 > G)) fail(PH_ERR_INVALID_ARGUMENT, "bad key shard");
  }
  if (dop == DENSE_LAYOUT) {
    ph_dense_layout& L = *dn->layout;
    L = ph_dense_layout{};
    L.num_groups = G;
    auto add = [&](int32_t per_group, int32_t op, int32_t bytes) {
      L.elems_per_group[L.num_tables] = per_group;
      L.reduce_op[L.num_tables] = op;
      L.elem_bytes[L.num_tables] = bytes;
      L.num_tables++;
    };
    add(1, PH_REDUCE_SUM_I64, 8);  // matched docs per group
    for (int j = 0; j < nvals; ++j) {
      if (val_ops[j] & 1) add(1, val_is_int[j] ? PH_REDUCE_SUM_I64 : PH_REDUCE_SUM_F64, 8);
      if (val_ops[j] & 2) add(1, PH_REDUCE_MIN_I64, 8);  // int64 values / order keys of doubles
      if (val_ops[j] & 4) add(1, PH_REDUCE_MAX_I64, 8);
    }
    if (num_hll) add(num_hll * m, PH_REDUCE_MAX_U32, 4);
    double bytes = 0;
    for (int t = 0; t < L.num_tables; ++t) bytes += (double)G * L.elems_per_group[t] * L.elem_bytes[t];
    if (bytes > kDenseTableBudget) fail(PH_ERR_UNSUPPORTED, "dense partials over a key space beyond the dense budget");
    return nullptr;
  }

  stamp("keys");
  // ---- kernel parameters
  KParams kp{};
  kp.num_vals = nvals;
  kp.num_hll = num_hll;
  kp.log2m = log2m ? log2m : 8;
  kp.num_groups = G;
  kp.num_group_cols = q->num_group_by;
  kp.docset = fds ? 1 : 0;
  {
    int64_t stride = 1;
    for (int g = 0; g < q->num_group_by; ++g) {
      kp.group_slot[g] = pl.slot.at(group_cols[g]);
      kp.group_stride[g] = stride;
      stride *= std::max<int64_t>(1, gdicts[g]->dict.size);
    }
  }
  for (int j = 0; j < nvals; ++j) {
    kp.val_ops[j] = val_ops[j];
    kp.val_is_int[j] = val_is_int[j];
    kp.val_op[j] = val_exprs[j];
  }
  for (int h = 0; h < num_hll; ++h) kp.hll_slot[h] = pl.slot.at(hll_cols[h]);

  // packed streams of the hot loop: slot 0 = the single-leaf filter column of each segment (if any),
  // then the group-by columns, then the aggregated value columns; all of them are LDS-staged.
  // FK_CONJ queries (a WHERE that is an AND of predicates, or of ORs of predicates on one column) instead get one
  // staged dictId stream per filter column and no per-segment filter slot, when they all fit kMaxStreams.
  std::vector<std::string> fcols;
  if (q->filter_root >= 0 && q->filter_nodes[q->filter_root].type == PH_FILTER_AND) {
    bool shape = true;
    const ph_filter_node& r = q->filter_nodes[q->filter_root];
    for (int i = 0; i < r.num_children && shape; ++i) {
      const ph_filter_node& k = q->filter_nodes[r.children[i]];
      std::string col;
      if (k.type == PH_FILTER_PREDICATE) {
        col = q->predicates[k.predicate].column;
      } else if (k.type == PH_FILTER_OR) {
        for (int j = 0; j < k.num_children && shape; ++j) {
          const ph_filter_node& g = q->filter_nodes[k.children[j]];
          if (g.type != PH_FILTER_PREDICATE) shape = false;
          else if (j == 0) col = q->predicates[g.predicate].column;
          else shape = col == q->predicates[g.predicate].column;
        }
      } else {
        shape = false;
      }
      if (shape && std::find(fcols.begin(), fcols.end(), col) == fcols.end()) fcols.push_back(col);
    }
    if (!shape || (int)fcols.size() > kMaxConj) fcols.clear();
  }
  std::vector<std::string> stream_cols;  // "" for the per-segment filter slot
  std::map<int, int> conj_stream;        // FK_CONJ: column slot -> staged stream
  auto stream_of = [&](const std::string& c, const char* kind) {
    std::string key = std::string(kind) + ":" + c;
    for (size_t i = 0; i < stream_cols.size(); ++i)
      if (stream_cols[i] == key) return (int)i;
    stream_cols.push_back(key);
    return (int)stream_cols.size() - 1;
  };
  auto assign_streams = [&](bool conj) {
    stream_cols.clear();
    conj_stream.clear();
    if (q->filter_root >= 0 && !conj) stream_cols.push_back("");
    for (int g = 0; g < q->num_group_by; ++g) kp.g_stream[g] = stream_of(group_cols[g], "id");
    for (int j = 0; j < nvals; ++j) {
      kp.v_stream[j] = stream_of(val_cols[j], "val");
      kp.v2_stream[j] = val_exprs[j] ? stream_of(val_cols2[j], "val") : kp.v_stream[j];
    }
    for (auto& c : fcols)
      if (conj) conj_stream[pl.slot.at(c)] = stream_of(c, "id");
    return (int)stream_cols.size() <= kMaxStreams;
  };
  const bool conj_query = !fcols.empty() && assign_streams(true);
  if (!conj_query && !assign_streams(false)) fail(PH_ERR_UNSUPPORTED, "too many column streams in one query");
  kp.f_stream = 0;  // the per-segment filter slot (unused by FK_CONJ queries, which have none)
  kp.nstage = (int)stream_cols.size();  // <= kMaxStreams == kMaxStage: every stream is staged

  // value column encodings + the table-wide value range (partitioned records carry value - vmin)
  int64_t vmin = INT64_MAX, vmax = INT64_MIN;
  for (int j = 0; j < nvals; ++j)
    for (auto* s : segs) {
      Column& c = *s->columns.at(val_cols[j]);
      if (val_is_int[j] && !val_exprs[j] && c.cardinality > 0 && j == 0) {
        vmin = std::min(vmin, c.dict.ints.front());
        vmax = std::max(vmax, c.dict.ints.back());
      }
    }

  // |integer SUM| < 2^53 whenever max |value| x total docs is: then no group's double can be inexact and the
  // per-group precision check is skipped (only for a local execute; a finalised shard also holds other ranks)
  bool sum_bounded[kMaxVals] = {};
  for (int j = 0; j < nvals; ++j)
    if (val_is_int[j]) sum_bounded[j] = term_amax[j] * (double)stats.num_total_docs < 4503599627370496.0;  // 2^52

  int mode = -3;  // DENSE_FINALIZE: no scan
  float dev_ms = 0.f;
  // a plain group-by's scan completion, matched-doc count and limit flags are read at the compaction's sync
  // (one host round trip instead of three)
  const bool defer_sync = q->num_group_by > 0 && num_hll == 0 && dop != DENSE_EXECUTE && !fin;
  std::unique_ptr<PinnedBlock> dsc;  // pinned: matched total, then 3 words per limit segment
  // the fused AND walks' sums (pinned, stream b): read at the end of the call, so the result compaction and copies
  // on the main stream overlap the walks instead of waiting behind them
  std::unique_ptr<PinnedBlock> fused_blk;
  std::vector<int64_t> fused_docs;  // numDocs of each walk's segment
  auto finish_fused = [&]() {
    if (!fused_blk) return;
    PH_HIP_CHECK(hipStreamSynchronize(lane.lane->stream_b));
    const unsigned long long* o = fused_blk->as<unsigned long long>();
    for (size_t x = 0; x < fused_docs.size(); ++x) stats.num_entries_scanned_in_filter += fused_docs[x] - 1 + (int64_t)o[x];
    fused_blk.reset();
    stamp("stat walk (fused)");
  };
  size_t dsc_nlim = 0;
  bool timed = false;  // this call recorded ev_start / ev_stop (some chunk was scanned)
  // device time of the call: the scan launches (ev_start .. ev_stop, including a numGroupsLimit pass) + the
  // inverted-leaf bitmap build (ev_bm0 .. ev_bm1); read after a sync of the stream
  auto device_elapsed = [&]() {
    float a = 0.f, b = 0.f;
    if (timed) PH_HIP_CHECK(hipEventElapsedTime(&a, lane.lane->ev_start, lane.lane->ev_stop));
    if (bm_timed) PH_HIP_CHECK(hipEventElapsedTime(&b, lane.lane->ev_bm0, lane.lane->ev_bm1));
    return a + b;
  };
  int64_t TR = G;  // rows of the output tables: the key space, or the slots of the MODE_GROUP_HASH table
  unsigned long long* hkeys = nullptr;
  if (fin) {
    // the tables hold the (already reduced) key shard [g0, g1): layout order of ph_query_dense_layout
    int t = 0;
    kp.out_count = reinterpret_cast<unsigned long long*>(dn->tables[t++]);
    for (int j = 0; j < nvals; ++j) {
      if (val_ops[j] & 1) kp.out_sum[j] = dn->tables[t++];
      if (val_ops[j] & 2) kp.out_min[j] = reinterpret_cast<int64_t*>(dn->tables[t++]);
      if (val_ops[j] & 4) kp.out_max[j] = reinterpret_cast<int64_t*>(dn->tables[t++]);
    }
    if (num_hll) kp.out_hll = reinterpret_cast<uint32_t*>(dn->tables[t++]);
    stats.plan_mode = mode;
    res->mode = mode;
  } else {
  stamp("kparams");
  // ---- mode selection (LDS table offsets are relative to the end of the staging areas, fixed below)
  size_t lds_tables = 16;
  int rec64 = 0;
  kp.stage_off = 0;
  if (q->num_group_by == 0) {
    mode = (nvals == 0 && num_hll == 0) ? MODE_COUNT : MODE_AGG;
    kp.lds_hll_off = 0;
    lds_tables = (size_t)num_hll * (m ? m : 1) * 4 + 16;
  } else {
    kp.lds_cnt_off = 0;
    size_t off = G < (int64_t(1) << 24) ? ((size_t)G * 4 + 15) / 16 * 16 : SIZE_MAX / 2;
    for (int j = 0; j < nvals; ++j) {
      auto place = [&](int32_t& o) {
        o = (int32_t)std::min<size_t>(off, INT32_MAX);
        off += (size_t)G * 8;
        off = (off + 15) / 16 * 16;
      };
      if (val_ops[j] & 1) place(kp.lds_sum_off[j]);
      if (val_ops[j] & 2) place(kp.lds_min_off[j]);
      if (val_ops[j] & 4) place(kp.lds_max_off[j]);
    }
    kp.lds_hll_off = (int32_t)std::min<size_t>(off, INT32_MAX);
    off += (size_t)G * num_hll * (m ? m : 1) * 4;
    const bool part_ok = num_hll == 0 && nvals <= 1 && (nvals == 0 || (val_is_int[0] && !val_exprs[0] && vmax >= vmin &&
                                                                       (uint64_t)(vmax - vmin) < (1ull << 32))) &&
                         G <= ((int64_t)kPartMaxParts << kPartKeysLog2) && !any_limit &&
                         !ctx->has(OPT_DISABLE_PARTITION);
    // LDS-private tables up to 64 KiB; r2 measured 96 KiB tables (one workgroup per CU) slower than the HBM table
    // for selective filters (SSB Q2.1, 7000 keys x COUNT + SUM: 3.9 vs 3.2 ms; Q2.3 3.2 vs 1.6 ms)
    // Dense LDS tables up to 64 KiB (PH_LDS_TABLE_MAX: tuning knob).  r2: routing 32-64 KiB tables to the cached
    // HBM table instead did not speed up SSB Q3.1 / Q4.2 and made an unfiltered 4375-key group-by 22x slower
    // (38.8 vs 1.7 ms: the cache cannot hold every key, the rest pays device atomics)
    size_t lds_table_max = 64 * 1024;
    if (ctx->has(OPT_LDS_TABLE_MAX)) lds_table_max = (size_t)std::max<int64_t>(0, ctx->opt(OPT_LDS_TABLE_MAX));
    const bool cache_ok = num_hll == 0 && nvals <= 1 && !ctx->has(OPT_NO_GROUP_CACHE);
    if (off <= (cache_ok ? lds_table_max : (size_t)64 * 1024)) {
      mode = MODE_GROUP_LDS;
      lds_tables = off;
    } else if (part_ok && G >= 65536) {
      mode = MODE_PARTITION;
    } else {
      int nout = 1;  // 8-byte tables per group
      for (int j = 0; j < nvals; ++j) nout += __builtin_popcount(val_ops[j] & 7);
      const double bytes = (double)G * (8.0 * nout + 4.0 * num_hll * (m ? m : 1));
      if (bytes <= kDenseTableBudget) {
        mode = MODE_GROUP_GLOBAL;
        // per-workgroup LDS cache of the groups it meets (open addressing, 1024 slots): repeated keys aggregate in
        // LDS and reach the HBM table once per workgroup at the end; a key that finds no slot within 8 probes goes
        // straight to the HBM table.  Device atomics from 64 lanes at 64 scattered addresses are the slow part of
        // this mode (r2: SSB Q2.1, 7000 keys, 3.2 ms of which ~2.2 ms atomics)
        if (cache_ok && G < (int64_t)0xffffffffu) {
          const size_t S = G <= 65536 ? 2048 : 1024;
          size_t o = 0;
          kp.gc_key_off = (int32_t)o;
          o += 4 * S;
          kp.lds_cnt_off = (int32_t)o;
          o += 4 * S;
          for (int j = 0; j < nvals; ++j) {
            if (val_ops[j] & 1) { kp.lds_sum_off[j] = (int32_t)o; o += 8 * S; }
            if (val_ops[j] & 2) { kp.lds_min_off[j] = (int32_t)o; o += 8 * S; }
            if (val_ops[j] & 4) { kp.lds_max_off[j] = (int32_t)o; o += 8 * S; }
          }
          kp.gc_slots = (int32_t)S;
          lds_tables = o;
        }
      } else {
        // key space beyond the dense budget: open-addressing table over the keys that can occur -- at most one
        // per scanned doc -- with >= 2x slots (DictionaryBasedGroupKeyGenerator's map-based holders, :598/:778)
        // (DISTINCTCOUNTHLL: 2^log2m registers per slot, the ObjectGroupByResultHolder of HyperLogLogs)
        if (dop) fail(PH_ERR_UNSUPPORTED, "dense partials over a key space beyond the dense budget");
        // numGroupsLimit here runs optimistically only: the scan goes ahead without truncation and the call fails
        // UNSUPPORTED afterwards if the table ends up with `limit` keys or more (see the launch below)
        int64_t live_docs = 0;
        for (int i = 0; i < nseg; ++i)
          if (seg_live[i]) live_docs += segs[i]->num_docs;
        int64_t H = 1024;
        while (H < 2 * std::min<int64_t>(G, live_docs)) H <<= 1;
        if ((double)H * (8.0 * nout + 8.0 + 4.0 * num_hll * (m ? m : 1)) > kDenseTableBudget)
          fail(PH_ERR_UNSUPPORTED, "group-by hash table too large for HBM budget");
        mode = MODE_GROUP_HASH;
        TR = H;
        kp.num_groups = H;
        kp.hmask = H - 1;
      }
    }
  }

  stamp("mode");
  // ---- outputs (dense execute: the caller's tables, initialised here)
  auto out_table = [&](int& t, size_t bytes) -> void* {
    if (dop == DENSE_EXECUTE) return dn->tables[t++];
    return scratch.alloc<uint8_t>(bytes);
  };
  int tix = 0;
  const int64_t hll_words = TR * num_hll * (m ? m : 1);
  kp.out_count = reinterpret_cast<unsigned long long*>(out_table(tix, 8 * (size_t)TR));
  for (int j = 0; j < nvals; ++j) {
    if (val_ops[j] & 1) kp.out_sum[j] = out_table(tix, 8 * (size_t)TR);
    if (val_ops[j] & 2) kp.out_min[j] = reinterpret_cast<int64_t*>(out_table(tix, 8 * (size_t)TR));
    if (val_ops[j] & 4) kp.out_max[j] = reinterpret_cast<int64_t*>(out_table(tix, 8 * (size_t)TR));
  }
  if (mode == MODE_GROUP_HASH) {
    hkeys = scratch.alloc<unsigned long long>(TR);
    kp.hkeys = hkeys;
  }
  if (num_hll) kp.out_hll = reinterpret_cast<uint32_t*>(out_table(tix, 4 * (size_t)hll_words));
  // identities of every output table (again before a numGroupsLimit rescan)
  auto init_tables = [&]() {
    PH_HIP_CHECK(hipMemsetAsync(kp.out_count, 0, sizeof(unsigned long long) * TR, st));
    for (int j = 0; j < nvals; ++j) {
      if (val_ops[j] & 1) PH_HIP_CHECK(hipMemsetAsync(kp.out_sum[j], 0, 8 * TR, st));
      if (val_ops[j] & 2) launch_fill_i64(kp.out_min[j], INT64_MAX, TR, st);
      if (val_ops[j] & 4) launch_fill_i64(kp.out_max[j], INT64_MIN, TR, st);
    }
    if (hkeys) PH_HIP_CHECK(hipMemsetAsync(hkeys, 0xFF, 8 * TR, st));  // kHashEmpty
    if (num_hll) PH_HIP_CHECK(hipMemsetAsync(kp.out_hll, 0, 4 * hll_words, st));
  };
  init_tables();

  stamp("outputs");
  // ---- device segment table, programs, chunks
  std::vector<DevSegment> dsegs;
  std::vector<std::vector<PNode>> sp_nodes;  // per DevSegment: its sparse scan leaves (SparseShape::scans)
  std::vector<FilterInsn> all_insns;
  std::vector<Chunk> chunks;
  std::vector<std::pair<size_t, std::vector<uint32_t>>> payload_fix;  // global insn index -> payload
  std::vector<std::pair<size_t, int>> bitmap_fix;                     // global insn index -> bitmap leaf
  std::vector<std::pair<size_t, std::vector<uint32_t>>> fset_fix;     // segment index -> FK_SET bitset
  std::vector<std::pair<size_t, int>> fbitmap_fix;                    // segment index -> bitmap leaf
  std::vector<std::pair<size_t, std::vector<uint32_t>>> conj_set_fix; // segment index * kMaxConj + leaf -> bitset
  std::vector<FbJob> fb_jobs;                                          // statistic passes: leaf doc bitmaps
  std::vector<std::pair<size_t, int>> sbm_fix;                         // segment index * kSparseBitmaps + k -> bitmap leaf
  std::vector<std::pair<size_t, std::vector<uint32_t>>> srng_fix;     // same index -> (first, count) container ranges
  std::vector<std::pair<size_t, std::vector<uint32_t>>> ctab_fix;     // segment index -> container table (group_cont)
  std::vector<std::pair<size_t, std::vector<uint32_t>>> sset_fix;     // segment index * kMaxConj + k -> bitset
  // k_group_sparse: every live segment's filter is a sparse_shape AND whose bitmaps keep < 1/8 of the docs (the
  // leaves' densities multiplied: an independence estimate) -> gather the matched docs instead of streaming every
  // referenced column
  bool sparse_plan = false;
  if ((mode == MODE_GROUP_LDS || mode == MODE_GROUP_GLOBAL) && num_hll == 0 && nvals <= 1 && q->num_group_by > 0) {
    bool ok = true;
    double docs = 0, hits = 0;
    for (int i = 0; i < nseg && ok; ++i) {
      if (!seg_live[i]) continue;
      const SparseShape sh = sparse_shape(roots[i]);
      ok = sh.ok;
      const double n = (double)std::max<int64_t>(1, segs[i]->num_docs);
      double est = n;
      for (auto& g : sh.groups) {
        double d = 0;
        for (int b : g) d += leaf_docs_estimate(pl.bitmaps[b]) / n;
        est *= std::min(1.0, d);
      }
      for (const PNode* k : sh.scans) {  // uniform dictIds: matched ids / cardinality
        const double card = (double)std::max<int64_t>(1, segs[i]->columns.at(slot_names[k->col])->cardinality);
        double ids = k->op == OP_RANGE ? (double)k->len : 0.0;
        if (k->op == OP_SET)
          for (uint32_t w : k->set) ids += (double)__builtin_popcount(w);
        est *= std::min(1.0, ids / card);
      }
      hits += sh.ok ? est : 0;
      docs += (double)segs[i]->num_docs;
    }
    sparse_plan = ok && docs > 0 && hits * 8 < docs;
    if (ctx->has(OPT_GROUP_SPARSE)) sparse_plan = ok && docs > 0 && ctx->opt(OPT_GROUP_SPARSE) != 0;
  }
  // k_agg_sparse over ANDs of scan leaves only (register-direct leaves, then gathers of the matched docs' values):
  // aggregation-only queries whose every segment's AND keeps < 1/8 of the docs (same estimate as above)
  bool agg_conj = false;
  if (mode == MODE_AGG && nvals >= 1 && (nvals == 1 || std::none_of(val_exprs.begin(), val_exprs.end(), [](int x) { return x != 0; }))) {
    bool ok = true;
    double docs = 0, hits = 0;
    for (int i = 0; i < nseg && ok; ++i) {
      if (!seg_live[i]) continue;
      const SparseShape sh = sparse_shape(roots[i]);
      ok = sh.ok && sh.groups.empty();
      double est = (double)std::max<int64_t>(1, segs[i]->num_docs);
      for (const PNode* k : sh.scans) {
        const double card = (double)std::max<int64_t>(1, segs[i]->columns.at(slot_names[k->col])->cardinality);
        double ids = k->op == OP_RANGE ? (double)k->len : 0.0;
        if (k->op == OP_SET)
          for (uint32_t w : k->set) ids += (double)__builtin_popcount(w);
        est *= std::min(1.0, ids / card);
      }
      hits += ok ? est : 0;
      docs += (double)segs[i]->num_docs;
    }
    agg_conj = ok && docs > 0 && hits * 8 < docs;
    if (ctx->has(OPT_AGG_SPARSE)) agg_conj = ok && docs > 0 && ctx->opt(OPT_AGG_SPARSE) != 0;
  }
  std::vector<std::pair<int32_t, int32_t>> dseg_chunks;                // device segment -> its chunk range
  std::vector<int> dseg_src;                                           // device segment -> query segment index
  std::vector<std::pair<int32_t, int32_t>> seg_words;                  // device segment -> [first, end) words to scan
  for (int k = 0; k < 8; ++k) tacc[k] = 0;
  for (int i = 0; i < nseg; ++i) {
    if (!seg_live[i]) continue;
    auto tb = tnow();
    ph_segment* s = segs[i];
    DevSegment d{};
    d.num_docs = s->num_docs;
    if (fds) d.docset = reinterpret_cast<uint32_t*>(fds->words + fds->word_off[i]);
    const PNode& root = roots[i];
    const size_t si = dsegs.size();
    auto conj_leaf = [&](const PNode& k) {
      return k.kind == L_NODE && k.scan && (k.op == OP_RANGE || k.op == OP_SET) && conj_stream.count(k.col);
    };
    const bool single_conj = conj_query && conj_leaf(root);
    if (root.kind == L_ALL) {
      d.fkind = FK_ALL;
    } else if (single_conj || (conj_query && root.op == OP_AND && (int)root.kids.size() <= kMaxConj &&
                               std::all_of(root.kids.begin(), root.kids.end(), conj_leaf))) {
      d.fkind = FK_CONJ;
      d.nconj = single_conj ? 1 : (int32_t)root.kids.size();
      d.conj_nidx = single_conj ? 0 : root.stats_nidx;  // range-index leaves first (mark_apply_and's order)
      if (d.conj_nidx) progs[i].apply_and = true;
      for (int k = 0; k < d.nconj; ++k) {
        const PNode& leaf = single_conj ? root : root.kids[k];
        d.cstream[k] = conj_stream.at(leaf.col);
        // a set leaf carries no range (clen 0 marks it until its device bitset is attached below: the prefetch
        // order keys off it).  r3: a set merged from same-column EQ leaves kept the first leaf's [lo, lo + 1), so
        // with no numGroupsLimit pass forcing the gathering kernel, SSB Q3.3 / Q3.4 matched only that dictId
        d.clo[k] = leaf.op == OP_SET ? 0u : leaf.lo;
        d.clen[k] = leaf.op == OP_SET ? 0u : leaf.len;
        if (leaf.op == OP_SET) conj_set_fix.push_back({si * kMaxConj + k, leaf.set});
      }
    } else if (conj_query && root.scan) {
      fail(PH_ERR_INVALID_ARGUMENT, "scan leaf without a staged stream");  // not reached: every filter column has one
    } else if (root.op == OP_RANGE) {
      d.fkind = FK_RANGE;
      d.fslot = root.col;
      d.flo = root.lo;
      d.flen = root.len;
    } else if (root.op == OP_SET) {
      d.fkind = FK_SET;
      d.fslot = root.col;
      fset_fix.push_back({si, root.set});
    } else if (root.op == OP_BITMAP) {
      d.fkind = FK_BITMAP;
      fbitmap_fix.push_back({si, root.bitmap_leaf});
    } else if (root.op == OP_DOCRANGES && root.ranges.size() == 2) {
      d.fkind = FK_DOCRANGE;
      d.flo = (uint32_t)root.ranges[0];
      d.flen = (uint32_t)(root.ranges[1] - root.ranges[0] + 1);
    } else {
      d.fkind = FK_GENERIC;
      emit(root, progs[i]);
      if (progs[i].max_depth > kMaxStack || (int)progs[i].insns.size() > kMaxProg)
        fail(PH_ERR_UNSUPPORTED, "filter too large for the GPU program");
      for (auto& in : progs[i].insns)
        if ((in.op == OP_AND || in.op == OP_OR) && in.col > kMaxStack) fail(PH_ERR_UNSUPPORTED, "filter too wide");
      d.prog_off = (int32_t)all_insns.size();
      d.prog_len = (int32_t)progs[i].insns.size();
      for (auto& pp : progs[i].payloads) payload_fix.push_back({d.prog_off + pp.first, pp.second});
      for (auto& bb : progs[i].bitmap_refs) bitmap_fix.push_back({d.prog_off + bb.first, bb.second});
      all_insns.insert(all_insns.end(), progs[i].insns.begin(), progs[i].insns.end());
    }
    for (auto& ss : stat_segs) {  // the statistic's leaf programs (k_filter_bitmaps), <= kMaxFbProgs per job
      if (ss.qi != i) continue;
      ss.dseg = (int32_t)si;
      for (size_t l = 0; l < ss.leaves.size(); ++l) {
        if (fast_leaf(ss.leaves[l])) continue;
        if (ss.jobs.empty() || fb_jobs[ss.jobs.back()].nprog == kMaxFbProgs) {
          FbJob job{};
          job.seg = (int32_t)si;
          job.nwords = ((int64_t)s->num_docs + 63) / 64;
          ss.jobs.push_back(fb_jobs.size());
          fb_jobs.push_back(job);
        }
        FbJob& job = fb_jobs[ss.jobs.back()];
        SegProgram sp;
        emit(ss.leaves[l], sp);
        if (sp.max_depth > kMaxStack || (int)sp.insns.size() > kMaxProg) fail(PH_ERR_UNSUPPORTED, "filter too large");
        job.off[job.nprog] = (int32_t)all_insns.size();
        job.len[job.nprog] = (int32_t)sp.insns.size();
        job.row[job.nprog] = (int32_t)l;
        ++job.nprog;
        for (auto& pp : sp.payloads) payload_fix.push_back({all_insns.size() + pp.first, pp.second});
        for (auto& bb : sp.bitmap_refs) bitmap_fix.push_back({all_insns.size() + bb.first, bb.second});
        all_insns.insert(all_insns.end(), sp.insns.begin(), sp.insns.end());
      }
    }
    tadd(3, tb);
    tb = tnow();
    if (sparse_plan || agg_conj) {
      const SparseShape sh = sparse_shape(root);
      if (sp_nodes.size() <= (size_t)si) sp_nodes.resize((size_t)si + 1);
      for (const PNode* sc : sh.scans) sp_nodes[si].push_back(*sc);
      d.sp_reg = sh.groups.empty() ? 1 : 0;
      d.sp_nbm = 0;
      for (auto& g : sh.groups)
        for (size_t j = 0; j < g.size(); ++j) {
          d.sp_or[d.sp_nbm] = j > 0;
          sbm_fix.push_back({si * kSparseBitmaps + d.sp_nbm, g[j]});
          ++d.sp_nbm;
        }
      d.sp_nscan = (int32_t)sh.scans.size();
      d.sp_stats = root.op == OP_AND && root.stats_nscan > 0;
      for (int k = 0; k < d.sp_nscan; ++k) {
        const PNode& leaf = *sh.scans[k];
        d.sp_slot[k] = leaf.col;
        d.sp_lo[k] = leaf.op == OP_SET ? 0u : leaf.lo;
        d.sp_len[k] = leaf.op == OP_SET ? 0u : leaf.len;
        if (leaf.op == OP_SET) sset_fix.push_back({si * kMaxConj + k, leaf.set});
      }
    }
    tadd(4, tb);
    tb = tnow();
    for (size_t sl = 0; sl < slot_names.size(); ++sl) {
      Column& c = *s->columns.at(slot_names[sl]);
      DevColumn& dc = d.cols[sl];
      dc.fwd = c.d_fwd.as<uint32_t>();
      dc.bits = c.bits;
      dc.cardinality = c.cardinality;
      dc.values = c.d_values.ptr;
    }
    for (int g = 0; g < q->num_group_by; ++g)
      d.cols[kp.group_slot[g]].remap = segment_remap(ctx, *s, *s->columns.at(group_cols[g]), *gdicts[g]);
    for (int h = 0; h < num_hll; ++h)
      d.cols[kp.hll_slot[h]].hll = segment_hll_table(ctx, *s->columns.at(hll_cols[h]), log2m, st);
    for (int j = 0; j < nvals; ++j) {
      for (int o = 0; o < (val_exprs[j] ? 2 : 1); ++o) {
        Column& c = *s->columns.at(o ? val_cols2[j] : val_cols[j]);
        DevValCol& v = o ? d.vals2[j] : d.vals[j];
        const bool col_int = c.data_type == PH_INT || c.data_type == PH_LONG;
        if (col_int && ensure_value_stream(ctx, s, c, st)) {
          v.kind = VK_PACKED;
          v.fwd = c.d_vpacked->as<uint32_t>();
          v.bits = c.vbits;
          v.base = c.vbase;
        } else {
          v.kind = col_int ? VK_DICT_I64 : VK_DICT_F64;
          v.fwd = c.d_fwd.as<uint32_t>();
          v.bits = c.bits;
          v.table = c.d_values.ptr;
        }
        d.streams[o ? kp.v2_stream[j] : kp.v_stream[j]] = DevStream{v.fwd, v.bits, 0};
      }
    }
    for (int g = 0; g < q->num_group_by; ++g) {
      Column& c = *s->columns.at(group_cols[g]);
      d.streams[kp.g_stream[g]] = DevStream{c.d_fwd.as<uint32_t>(), c.bits, 0};
    }
    for (int k = 0; d.fkind == FK_CONJ && k < d.nconj; ++k) {
      Column& c = *s->columns.at(slot_names[(d.nconj == 1 && root.op != OP_AND) ? root.col : root.kids[k].col]);
      d.streams[d.cstream[k]] = DevStream{c.d_fwd.as<uint32_t>(), c.bits, 0};
    }
    if (q->filter_root >= 0 && !conj_query) {
      // bits = 0: nothing to stage for this segment's filter (FK_ALL / bitmap / doc range / program)
      d.streams[0] = DevStream{nullptr, 0, 0};
      if (d.fkind == FK_RANGE || d.fkind == FK_SET) {
        Column& c = *s->columns.at(slot_names[d.fslot]);
        d.streams[0] = DevStream{c.d_fwd.as<uint32_t>(), c.bits, 0};
      }
    }
    // chunks cover only the words the filter can match in (SortedIndexBasedFilterOperator: a sorted leaf, alone
    // or under an AND, bounds the docs; r1 staged every stream of the whole segment)
    tadd(5, tb);
    tb = tnow();
    const std::pair<int64_t, int64_t> span = doc_span(root, s->num_docs);
    seg_words.push_back({(int32_t)(span.first / 64), (int32_t)((span.second + 63) / 64)});
    dseg_src.push_back(i);
    dsegs.push_back(d);
    stats.num_segments_matched++;
    tadd(6, tb);
  }
  if (host_times)
    fprintf(stderr, "[ph host]   segtable: filter+stat %.3f sparse %.3f columns %.3f span+push %.3f ms\n", tacc[3], tacc[4],
            tacc[5], tacc[6]);
  // selective inverted-index leaves (k_agg_sparse): every segment's filter is one bitmap leaf and together they
  // match < 1/8 of the docs -> gather the matched docs' values instead of streaming the columns.  Decided before the
  // chunk list: the container form replaces it (r6: config 5's 400 segments built 244K streaming chunks, 0.25 ms of
  // host time, only to drop them)
  bool all_bitmap_agg = mode == MODE_AGG && !dsegs.empty();
  for (int j = 0; j < nvals; ++j) all_bitmap_agg = all_bitmap_agg && !val_exprs[j];
  for (auto& d : dsegs) all_bitmap_agg = all_bitmap_agg && d.fkind == FK_BITMAP;
  bool agg_sparse_plan = agg_conj;
  {
    int64_t docs = 0, hits = 0;
    if (all_bitmap_agg) {
      for (auto& d : dsegs) docs += d.num_docs;
      for (auto& fb : fbitmap_fix) hits += (int64_t)leaf_docs_estimate(pl.bitmaps[fb.second]);
    }
    agg_sparse_plan = (all_bitmap_agg && hits * 8 < docs) || agg_conj;
    if (ctx->has(OPT_AGG_SPARSE)) agg_sparse_plan = (all_bitmap_agg || agg_conj) && ctx->opt(OPT_AGG_SPARSE) != 0;
  }
  const bool agg_cont_plan = cont_defer && agg_sparse_plan && all_bitmap_agg && !agg_conj;
  int64_t chunk_docs_total = 0;  // the streaming chunk list's words x 64 and its widest chunk
  int32_t chunk_words_max = 0;
  if (agg_cont_plan) {
    dseg_chunks.assign(seg_words.size(), {0, 0});
  } else {
    // chunk size: 16384 docs, smaller when the whole scan has too few chunks to give every CU several (a single
    // 10M-row segment clipped to an 8 % sorted range is ~50 full chunks: latency-bound on 50 workgroups)
    int64_t total_words = 0;
    for (auto& sw : seg_words) total_words += std::max(0, sw.second - sw.first);
    const int32_t cw = (int32_t)std::max<int64_t>(
        32, std::min<int64_t>(kChunkWords, (total_words + 4 * ctx->num_cus - 1) / (4 * ctx->num_cus)));
    size_t nch = 0;
    for (auto& sw : seg_words) nch += (size_t)((std::max(0, sw.second - sw.first) + cw - 1) / cw);
    chunks.reserve(nch);
    dseg_chunks.reserve(seg_words.size());
    for (size_t si = 0; si < seg_words.size(); ++si) {
      dseg_chunks.push_back({(int32_t)chunks.size(), 0});
      for (int32_t w = seg_words[si].first; w < seg_words[si].second; w += cw)
        chunks.push_back({(int32_t)si, w, std::min(seg_words[si].second, w + cw), 0});
      dseg_chunks.back().second = (int32_t)chunks.size();
    }
    chunk_docs_total = total_words * 64;
    chunk_words_max = (int32_t)std::min<int64_t>(cw, total_words);
  }
  stamp("segtable");
  // ---- per-wave staging layout: one span per staged stream, sized by its widest segment; the tile is the
  // largest (<= 32 words) whose spans fit the kernel's prefetch register pool
  {
    int maxbits[kMaxStage] = {};
    for (int s = 0; s < kp.nstage; ++s)
      for (auto& d : dsegs) maxbits[s] = std::max(maxbits[s], (int)d.streams[s].bits);
    const int pool = mode == MODE_COUNT ? kPrefetchCount : (mode == MODE_PARTITION ? kPrefetchPartition : kPrefetchOther);
    // r1/r2 sweeps: MODE_PARTITION rounds (8 waves x 8 words) append ~2048 records, which keeps a
    // partition's ring (32 slots) from overflowing
    // (r2 interleaved sweep, config 3: partition tiles of 12 words 3.80-3.82 ms, 8 words 3.89-3.93, 10 words 4.36)
    int tw = mode == MODE_PARTITION ? 12 : ((mode == MODE_GROUP_LDS || kp.gc_slots) ? 16 : kMaxTileWords);
    if (ctx->has(OPT_TILE_WORDS)) tw = (int)std::max<int64_t>(4, std::min<int64_t>(kMaxTileWords, ctx->opt(OPT_TILE_WORDS)));
    auto loads = [&](int t) {
      int n = 0;
      for (int s = 0; s < kp.nstage; ++s) n += maxbits[s] ? stage_loads(t, maxbits[s]) : 0;
      return n;
    };
    while (tw > 4 && loads(tw) > pool) tw /= 2;
    if (mode == MODE_GROUP_LDS) {  // staging + the LDS tables within one CU's 160 KiB
      auto stage = [&](int t) {
        size_t b = 0;
        for (int s2 = 0; s2 < kp.nstage; ++s2) b += maxbits[s2] ? stage_stream_bytes(t, maxbits[s2]) : 0;
        return (size_t)kWaves * std::max<size_t>(16, b);
      };
      while (tw > 4 && stage(tw) + lds_tables > 160 * 1024) tw /= 2;
      if (stage(tw) + lds_tables > 160 * 1024) fail(PH_ERR_UNSUPPORTED, "LDS group table and staging exceed 160 KiB");
    }
    if (loads(tw) > pool) fail(PH_ERR_UNSUPPORTED, "staged streams too wide for the prefetch pool");
    kp.tile_words = tw;
    int32_t soff = 0;
    for (int s = 0; s < kp.nstage; ++s) {
      kp.stage_soff[s] = soff;
      soff += maxbits[s] ? stage_stream_bytes(tw, maxbits[s]) : 0;
    }
    kp.stage_stride = std::max<int32_t>(16, soff);
  }
  // a decode that gathers (bitset / bitmap / program filters, key remaps, dictionary values, HLL tables)
  // would wait behind an early prefetch
  for (auto& d : dsegs) {
    bool g = d.fkind == FK_SET || d.fkind == FK_BITMAP || d.fkind == FK_GENERIC || num_hll > 0;
    for (int k = 0; d.fkind == FK_CONJ && k < d.nconj; ++k) g |= d.cset[k] != nullptr || d.clen[k] == 0;
    for (int gi = 0; gi < q->num_group_by; ++gi) g |= d.cols[kp.group_slot[gi]].remap != nullptr;
    for (int j = 0; j < nvals; ++j) g |= d.vals[j].kind != VK_PACKED || (val_exprs[j] && d.vals2[j].kind != VK_PACKED);
    if (g && mode != MODE_COUNT) kp.late_prefetch = 1;
    if (g && mode == MODE_COUNT && d.fkind != FK_RANGE && d.fkind != FK_ALL && d.fkind != FK_DOCRANGE) kp.late_prefetch = 1;
  }
  // numGroupsLimit: every segment that may reach the limit gets a keep bitset over the global keys (filled by
  // the first-seen pass below, read by the scan: a gather, so the late prefetch)
  std::vector<int> limit_segs;
  unsigned long long* limit_scal = nullptr;  // [3] per limit segment: distinct, threshold, reached
  uint32_t* limit_keep = nullptr;             // [limit segments][ceil(G / 32)] keep bitsets
  uint32_t* limit_first = nullptr;            // [limit segments][G] first matching doc per key
  const int base_late = kp.late_prefetch;     // the scan's prefetch order without the keep-bitset gathers
  // numGroupsLimit, optimistic form: scan without truncation first; only when the merged table then holds >= limit
  // keys can a segment have reached the limit, and only then do the first-seen pass and the truncating rescan run
  // (r2 ran the pass whenever a segment's cardinality product reached the limit: SSB Q3.2-Q4.3, products of
  // 0.4-1.75M keys over a few hundred real groups).  PH_LIMIT_EAGER=1 restores the pass-first order (tests).
  const bool limit_opt = !ctx->has(OPT_LIMIT_EAGER) || mode == MODE_GROUP_HASH;
  if (any_limit && q->num_group_by > 0) {
    for (size_t k = 0; k < dsegs.size(); ++k)
      if (seg_limit[dseg_src[k]]) limit_segs.push_back((int)k);
  }
  if (!limit_segs.empty() && mode != MODE_GROUP_HASH) {
    const double keep_bytes = (double)limit_segs.size() * (double)((G + 31) / 32) * 4.0;
    if (keep_bytes > 8e9) fail(PH_ERR_UNSUPPORTED, "numGroupsLimit emulation needs too many key bitsets");
    // one block each for the limit segments' keep bitsets and first-doc tables (every segment's pass runs in one
    // launch, the selections in one launch per step)
    const double first_bytes = (double)limit_segs.size() * (double)G * 4.0;
    if (first_bytes > 16e9) fail(PH_ERR_UNSUPPORTED, "numGroupsLimit emulation needs too many first-doc tables");
    const size_t kw = (size_t)(G + 31) / 32;
    limit_keep = scratch.alloc<uint32_t>(std::max<size_t>(1, kw * limit_segs.size()));
    limit_first = scratch.alloc<uint32_t>(std::max<size_t>(1, (size_t)G * limit_segs.size()));
    for (size_t t = 0; t < limit_segs.size(); ++t) {
      dsegs[limit_segs[t]].keep = limit_keep + t * kw;
      dsegs[limit_segs[t]].first_doc = limit_first + t * (size_t)G;
    }
    limit_scal = scratch.alloc<unsigned long long>(3 * limit_segs.size());
    if (!limit_segs.empty()) PH_HIP_CHECK(hipMemsetAsync(limit_scal, 0, 24 * limit_segs.size(), st));
    if (!limit_segs.empty()) kp.late_prefetch = 1;
  }
  {
    // the matched-doc total and the applyAnd entry count: one zeroed 16-byte block (one fill, not two)
    bool apply_and = false;
    for (size_t i = 0; i < progs.size(); ++i) apply_and |= seg_live[i] && progs[i].apply_and;
    if (q->num_group_by > 0 || apply_and) {
      unsigned long long* sc = scratch.alloc<unsigned long long>(2);
      PH_HIP_CHECK(hipMemsetAsync(sc, 0, 16, st));
      if (q->num_group_by > 0) kp.matched_total = sc;
      if (apply_and) kp.filter_entries = sc + 1;
    }
  }
  // per-segment tile pieces: the 1 KiB wave-loads of a full tile, stream by stream
  for (auto& d : dsegs) fill_tile_pieces(d, kp.nstage, kp.stage_soff, kp.tile_words);
  // the lean kernel A (k_part_scan) covers gather-free tiles with ALL / RANGE / DOCRANGE filter leaves
  kp.part_fast = !kp.late_prefetch && !ctx->has(OPT_PART_GENERIC);
  for (auto& d : dsegs)
    if (d.fkind != FK_ALL && d.fkind != FK_RANGE && d.fkind != FK_DOCRANGE) kp.part_fast = 0;
  // the lean aggregation kernel (k_agg_lean) covers one packed integer value column with ALL / RANGE / DOCRANGE
  // leaves; its 32-bit tile sums need value offsets below 2^26
  //   r3: also FK_CONJ ANDs of range leaves (no applyAnd statistic to count) and integer 2-operand value terms of
  //   two packed columns (per-doc int64 fold; SSB Q1.x)
  kp.agg_fast = mode == MODE_AGG && nvals == 1 && num_hll == 0 && val_is_int[0] && !kp.late_prefetch &&
                !ctx->has(OPT_AGG_GENERIC);
  for (auto& d : dsegs) {
    if (!kp.agg_fast) break;  // (val_exprs is empty without value columns)
    bool conj_ok = d.fkind == FK_CONJ && d.conj_nidx == 0;
    for (int k = 0; conj_ok && k < d.nconj; ++k) conj_ok = d.cset[k] == nullptr && d.clen[k] > 0;
    if ((d.fkind != FK_ALL && d.fkind != FK_RANGE && d.fkind != FK_DOCRANGE && !conj_ok) ||
        d.vals[0].kind != VK_PACKED || (!val_exprs[0] && d.streams[kp.v_stream[0]].bits > 26) ||
        (val_exprs[0] && d.vals2[0].kind != VK_PACKED))
      kp.agg_fast = 0;
  }
  // the lean LDS group-by (k_group_lds_lean): identity remaps, at most one packed integer value column whose
  // offsets from the table-wide minimum fit 32 bits, ALL / RANGE / DOCRANGE leaves
  kp.lds_fast = mode == MODE_GROUP_LDS && num_hll == 0 && nvals <= 1 && !kp.late_prefetch &&
                !ctx->has(OPT_LDS_GENERIC);
  if (nvals == 1)
    kp.lds_fast = kp.lds_fast && val_is_int[0] && !val_exprs[0] && vmax >= vmin && (uint64_t)(vmax - vmin) < (1ull << 32);
  for (auto& d : dsegs)
    if ((d.fkind != FK_ALL && d.fkind != FK_RANGE && d.fkind != FK_DOCRANGE) ||
        (nvals == 1 && d.vals[0].kind != VK_PACKED))
      kp.lds_fast = 0;
  stamp("staging");
  // the k_agg_sparse plan decided above
  {
    kp.agg_sparse = agg_sparse_plan;
    if (kp.agg_sparse) kp.agg_fast = 0;
    kp.agg_cont = agg_cont_plan;
    if (kp.agg_cont) {
      // chunks = ranges of <= 8 containers of each dictId of each segment's leaf (a wave takes one at a time)
      chunks.clear();
      for (auto& fb : fbitmap_fix) {
        const BitmapLeaf& bl = pl.bitmaps[fb.second];
        const Column& col = *bl.col;
        DevSegment& d = dsegs[fb.first];
        d.cdir = col.d_dir.as<RoaringContainer>();
        d.cbase = col.d_inverted.as<uint8_t>();
        dseg_chunks[fb.first].first = (int32_t)chunks.size();
        for (int32_t id : bl.dict_ids) {
          const int64_t f = col.dir_begin[id], e = col.dir_begin[id + 1];
          for (int64_t x = f; x < e; x += 8)
            chunks.push_back({(int32_t)fb.first, (int32_t)x, (int32_t)std::min<int64_t>(e, x + 8), 0});
        }
        dseg_chunks[fb.first].second = (int32_t)chunks.size();
      }
    }
  }
  stamp("sparse");
  // the register-direct leaves' loads per lane (conj_reg.h): by the widest scan column of an sp_reg segment
  // (2: every leaf <= 8 bits, all loads hoisted; 0: no segment has register-direct leaves)
  kp.sparse_c = 0;
  for (auto& d : dsegs)
    for (int k = 0; d.sp_reg && k < d.sp_nscan; ++k)
      kp.sparse_c = std::max(kp.sparse_c, d.cols[d.sp_slot[k]].bits > 16 ? 8 : d.cols[d.sp_slot[k]].bits > 8 ? 4 : 2);
  // r6: the all-leaves-at-once form (C = 2, every leaf <= 8 bits) holds 185 VGPRs (2 waves per SIMD); leaf by leaf
  // (C = 4, 139 VGPRs) measured 13.33 vs 13.89 ms of kernels on the scan-dimension SSB flight (Q2.1 1.02 vs 1.16), the
  // same on Q1.x -- so it is the default; option sparse_c = 2 restores the wide form
  if (kp.sparse_c == 2) kp.sparse_c = 4;
  if (kp.sparse_c > 0 && ctx->has(OPT_SPARSE_C)) {
    const int64_t c = ctx->opt(OPT_SPARSE_C);
    bool narrow = true;  // the wide form needs every leaf <= 8 bits
    for (auto& d : dsegs)
      for (int k = 0; d.sp_reg && k < d.sp_nscan; ++k) narrow = narrow && d.cols[d.sp_slot[k]].bits <= 8;
    if (c <= 2 && narrow) kp.sparse_c = 2;
    else kp.sparse_c = std::max(kp.sparse_c, c >= 8 ? 8 : 4);
  }
  // the register-direct COUNT (k_count_reg): every segment a dictId RANGE scan leaf, everything, or a sorted range
  if (mode == MODE_COUNT && !kp.late_prefetch && !ctx->has(OPT_COUNT_GENERIC)) {
    int fb = 1;
    bool ok = true;
    for (auto& d : dsegs) {
      ok = ok && (d.fkind == FK_RANGE || d.fkind == FK_ALL || d.fkind == FK_DOCRANGE);
      if (d.fkind == FK_RANGE) fb = std::max(fb, (int)d.streams[kp.f_stream].bits);
    }
    if (ok && fb <= 32) kp.count_reg = (fb + 3) / 4;
  }
  const size_t stage_bytes = (size_t)(mode == MODE_PARTITION ? kPartWaves : kWaves) * kp.stage_stride;
  size_t lds = 0;
  if (mode == MODE_PARTITION) {
    lds = 0;  // laid out with the partition parameters below
  } else {
    kp.stage_off = 0;
    kp.lds_cnt_off += (int32_t)stage_bytes;
    kp.lds_hll_off += (int32_t)stage_bytes;
    kp.gc_key_off += (int32_t)stage_bytes;
    for (int j = 0; j < nvals; ++j) {
      kp.lds_sum_off[j] += (int32_t)stage_bytes;
      kp.lds_min_off[j] += (int32_t)stage_bytes;
      kp.lds_max_off[j] += (int32_t)stage_bytes;
    }
    lds = stage_bytes + lds_tables;
    kp.pl_misc_off = 0;
    if (kp.lds_fast) {
      // table copies (one per wave when they fit in 48 KiB); COUNT+SUM packed in one 64-bit word when a copy's
      // docs (bounded by its workgroup's) keep count < 2^24 and the offset sum < 2^40
      int32_t mcw = 1;
      for (auto& ch : chunks) mcw = std::max(mcw, ch.word_end - ch.word_begin);
      const uint64_t vrange = nvals ? (uint64_t)(vmax - vmin) : 0;
      auto layout = [&](bool pack) {
        kp.lds_copy_bytes = (int32_t)(((size_t)G * (pack ? 16 : 20) + 15) / 16 * 16);
        kp.lds_copies = (size_t)kWaves * kp.lds_copy_bytes <= 48 * 1024 ? kWaves : 1;
        return stage_bytes + (size_t)kp.lds_copies * kp.lds_copy_bytes;
      };
      size_t l = layout(true);
      const int bpc = std::min<int>(4, (int)std::max<size_t>(1, (160 * 1024) / l));
      const int64_t grid_est = std::max<int64_t>(1, std::min<int64_t>((int64_t)chunks.size(), (int64_t)ctx->num_cus * bpc));
      const double wg_docs = (double)((int64_t)chunks.size() + grid_est - 1) / grid_est * mcw * 64.0;
      kp.lds_pack = wg_docs < 16777216.0 && wg_docs * (double)vrange < 1099511627776.0;
      if (!kp.lds_pack) l = layout(false);
      kp.part_vbase = nvals ? vmin : 0;
      if ((size_t)kp.lds_copy_bytes > 64 * 1024) kp.lds_fast = 0;  // not expected: G is an LDS-sized key space
      else lds = std::max(lds, l);
      // the register-direct form (k_group_reg): <= 2 group columns of <= 16 bits, filter streams <= 32 bits, value
      // streams <= 32 bits, the packed slot words, and a lane-interleaved table (L slots per key) in <= 40 KiB so
      // that four workgroups share a CU (r3, config3-lds: L = 16 at four workgroups per CU 1.08 ms, L = 32 at
      // three 1.18-1.24 ms -- occupancy beats the 2-way bank sharing of L = 16)
      if (kp.lds_fast && kp.lds_pack && q->num_group_by <= 2 && !ctx->has(OPT_LDS_LEAN)) {
        int fb = 1, gb = 1, vb = 1;
        for (auto& d : dsegs) {
          if (d.fkind == FK_RANGE) fb = std::max(fb, (int)d.streams[kp.f_stream].bits);
          for (int g = 0; g < q->num_group_by; ++g) gb = std::max(gb, (int)d.streams[kp.g_stream[g]].bits);
          if (nvals) vb = std::max(vb, (int)d.streams[kp.v_stream[0]].bits);
        }
        const int cf = fb <= 12 ? 3 : 8, cg = gb <= 8 ? 2 : 4, cv = nvals ? (vb <= 16 ? 4 : 8) : 0;
        constexpr size_t kRegTableBytes = 40 * 1024;
        int lg = 5;
        if (ctx->has(OPT_GROUP_REG_LG)) lg = (int)std::max<int64_t>(0, std::min<int64_t>(5, ctx->opt(OPT_GROUP_REG_LG)));
        while (lg > 0 && (size_t)(G + 1) * 16 << lg > kRegTableBytes) --lg;  // + the dummy row of missed docs
        if (fb <= 32 && gb <= 16 && vb <= 32 && (size_t)(G + 1) * 16 << lg <= kRegTableBytes &&
            cf + q->num_group_by * cg + cv <= 20) {
          kp.group_reg = 1;
          kp.group_reg_lanes_log2 = lg;
          kp.group_reg_cf = cf;
          kp.group_reg_cg = cg;
          kp.group_reg_cv = cv;
          lds = (size_t)(G + 1) * 16 << lg;
        }
      }
    }
    if (sparse_plan) {  // the generic tables (LDS table or group cache) + one matched-doc list per wave
      kp.pl_misc_off = (int32_t)((stage_bytes + lds_tables + 15) / 16 * 16);  // after the generic layout
      // + the staged scan-leaf sets when a segment has register-direct leaves (4 KiB: it can cost a bitmap-only
      // plan its LDS fit)
      const size_t l2 = (size_t)kp.pl_misc_off + (size_t)kWaves * kSparseStepWords * 64 * sizeof(uint16_t) +
                        (kp.sparse_c ? (size_t)kMaxConj * kConjSetWords * sizeof(uint32_t) : 0);
      if (l2 <= 160 * 1024) {
        kp.group_sparse = 1;
        kp.group_reg = 0;
        lds = l2;
      }
    }
    if (kp.agg_sparse) {  // no staging: the HLL registers and one matched-doc list (uint16 offsets) per wave
      kp.lds_hll_off = 0;
      kp.pl_misc_off = (int32_t)(((size_t)num_hll * (m ? m : 1) * 4 + 16 + 15) / 16 * 16);
      lds = (size_t)kp.pl_misc_off + (size_t)kWaves * kSparseStepWords * 64 * sizeof(uint16_t) +
            (kp.sparse_c ? (size_t)kMaxConj * kConjSetWords * sizeof(uint32_t) : 0);
    }
    if (gs_defer) {
      // k_group_sparse from the containers: no filter-statistic pass may need the doc bitmaps (a numGroupsLimit
      // first-seen pass, which runs the generic program, builds them when it runs: late_bitmaps)
      int max_nbm = 1;
      for (auto& d : dsegs) max_nbm = std::max(max_nbm, (int)d.sp_nbm);
      const size_t cbm = (size_t)max_nbm * kContWords * 8;
      const size_t off = (lds + 15) / 16 * 16;
      kp.group_cont = kp.group_sparse && stat_segs.empty() && off + cbm <= 160 * 1024;
      if (kp.group_cont) {
        kp.cont_bm_off = (int32_t)off;
        lds = off + cbm;
        // chunks of whole 65536-doc container keys (kContWords words): one LDS build per key and leaf
        chunks.clear();
        for (size_t si = 0; si < dsegs.size(); ++si) {
          const int32_t nw = (int32_t)((dsegs[si].num_docs + 63) / 64);
          dseg_chunks[si].first = (int32_t)chunks.size();
          for (int32_t w = 0; w < nw; w += kContWords) chunks.push_back({(int32_t)si, w, std::min(nw, w + kContWords), 0});
          dseg_chunks[si].second = (int32_t)chunks.size();
        }
        // leaf k of a segment: its dictIds' container ranges (uploaded with the predicate payloads)
        for (auto& sb : sbm_fix) {
          const BitmapLeaf& bl = pl.bitmaps[sb.second];
          DevSegment& d = dsegs[sb.first / kSparseBitmaps];
          const int k = (int)(sb.first % kSparseBitmaps);
          d.sp_cdir[k] = bl.col->d_dir.as<RoaringContainer>();
          d.sp_cbase[k] = bl.col->d_inverted.as<uint8_t>();
          std::vector<uint32_t> rg;
          for (int32_t id : bl.dict_ids) {
            const int64_t f = bl.col->dir_begin[id], n = bl.col->dir_begin[id + 1] - f;
            if (n > 0) {
              rg.push_back((uint32_t)f);
              rg.push_back((uint32_t)n);
            }
          }
          d.sp_nrng[k] = (int32_t)(rg.size() / 2);
          srng_fix.push_back({sb.first, std::move(rg)});
        }
        // per segment: [65536-doc key][range t over its leaves] -> the range's container of that key (or -1), so
        // the kernel indexes the directory instead of searching it
        std::vector<std::vector<std::pair<const Column*, std::pair<int64_t, int64_t>>>> segr(dsegs.size());
        for (auto& sb : sbm_fix) {
          const BitmapLeaf& bl = pl.bitmaps[sb.second];
          for (int32_t id : bl.dict_ids) {
            const int64_t f = bl.col->dir_begin[id], e = bl.col->dir_begin[id + 1];
            if (e > f) segr[sb.first / kSparseBitmaps].push_back({bl.col, {f, e}});
          }
        }
        for (size_t si = 0; si < dsegs.size(); ++si) {
          const size_t ntot = segr[si].size(), nkeys = ((size_t)dsegs[si].num_docs + 65535) / 65536;
          std::vector<uint32_t> tab(std::max<size_t>(1, nkeys * ntot), 0xffffffffu);
          for (size_t t = 0; t < ntot; ++t) {
            const Column* col = segr[si][t].first;
            for (int64_t x = segr[si][t].second.first; x < segr[si][t].second.second; ++x) {
              const size_t key = (size_t)col->dir[x].key;
              if (key < nkeys) tab[key * ntot + t] = (uint32_t)x;
            }
          }
          dsegs[si].sp_ntot = (int32_t)ntot;
          ctab_fix.push_back({si, std::move(tab)});
        }
      }
    }
    // 160 KiB of LDS per CU (gfx950); HLL registers of a large log2m do not fit beside the staging areas
    if (lds > 160 * 1024) fail(PH_ERR_UNSUPPORTED, "aggregation state exceeds the LDS of one CU (HLL log2m too large)");
  }
  // the deferred doc bitmaps, when neither container plan was taken (any mode: the plans that read them)
  if ((cont_defer || gs_defer) && !kp.agg_cont && !kp.group_cont) {
    PH_HIP_CHECK(hipEventRecord(lane.lane->ev_bm0, st));
    build_bitmaps();
    PH_HIP_CHECK(hipEventRecord(lane.lane->ev_bm1, st));
    bm_timed = true;
  }
  // every predicate payload (program sets / ranges, FK_SET / FK_CONJ / sparse-leaf bitsets) in ONE upload: r4 issued
  // one small copy per payload (SSB Q3.3 on 60 segments: 120 copies, ~1 ms of setup)
  {
    std::vector<uint32_t> blob;
    std::vector<size_t> at;
    auto put = [&](const std::vector<uint32_t>& w) {
      at.push_back(blob.size());
      blob.insert(blob.end(), w.begin(), w.end());
      blob.resize((blob.size() + 4) & ~(size_t)3, 0u);  // >= 1 word of pad, 16-byte aligned starts
    };
    for (auto& pf : payload_fix) put(pf.second);
    for (auto& ff : fset_fix) put(ff.second);
    for (auto& sf : sset_fix) put(sf.second);
    for (auto& cf : conj_set_fix) put(cf.second);
    for (auto& rf : srng_fix) put(rf.second);
    for (auto& tf : ctab_fix) put(tf.second);
    if (!blob.empty()) {
      uint32_t* dblob = scratch.alloc<uint32_t>(blob.size());
      // from pinned staging (slot 2): no host wait for the copy (r5: a pageable copy here synchronised the stream,
      // so the host waited for the bitmap build before it could finish the setup)
      uint32_t* hblob = static_cast<uint32_t*>(lane.lane->host_staging(4 * blob.size(), 2));
      memcpy(hblob, blob.data(), 4 * blob.size());
      PH_HIP_CHECK(hipMemcpyAsync(dblob, hblob, 4 * blob.size(), hipMemcpyHostToDevice, st));
      size_t i = 0;
      for (auto& pf : payload_fix) all_insns[pf.first].ptr = dblob + at[i++];
      for (auto& ff : fset_fix) dsegs[ff.first].fptr = dblob + at[i++];
      for (auto& sf : sset_fix) dsegs[sf.first / kMaxConj].sp_set[sf.first % kMaxConj] = dblob + at[i++];
      for (auto& cf : conj_set_fix) dsegs[cf.first / kMaxConj].cset[cf.first % kMaxConj] = dblob + at[i++];
      for (auto& rf : srng_fix)
        dsegs[rf.first / kSparseBitmaps].sp_rng[rf.first % kSparseBitmaps] = reinterpret_cast<const RoaringRange*>(dblob + at[i++]);
      for (auto& tf : ctab_fix) dsegs[tf.first].sp_ctab = reinterpret_cast<const int32_t*>(dblob + at[i++]);
    }
  }
  for (auto& bf : bitmap_fix) all_insns[bf.first].ptr = bitmap_dev[bf.second];
  for (auto& fb : fbitmap_fix) dsegs[fb.first].fptr = bitmap_dev[fb.second];
  for (auto& sb : sbm_fix) dsegs[sb.first / kSparseBitmaps].sp_bm[sb.first % kSparseBitmaps] = bitmap_dev[sb.second];
  // ANDs of scans on the register-direct sparse front end: its leaf masks become the statistic's leaf bitmaps
  // (conj_reg.h conj_leaf_out), one buffer for all of them (their walks run after the scan, on stream b)
  if ((kp.group_sparse || kp.agg_sparse) && kp.sparse_c > 0 && !ctx->has(OPT_STAT_FUSE)) {
    auto same = [](const PNode& a, const PNode& b) {
      return a.col == b.col && a.op == b.op && a.lo == b.lo && a.len == b.len && a.set == b.set;
    };
    size_t words = 0;
    std::vector<std::pair<size_t, std::vector<int>>> plan;  // (stat seg, sparse leaf of each stat leaf)
    for (size_t t = 0; t < stat_segs.size(); ++t) {
      StatSeg& ss = stat_segs[t];
      if (ss.kind != ST_SCANAND || ss.dseg < 0 || !dsegs[ss.dseg].sp_reg) continue;
      if ((size_t)ss.dseg >= sp_nodes.size()) continue;
      const std::vector<PNode>& sp = sp_nodes[ss.dseg];
      if (sp.size() != ss.leaves.size()) continue;
      std::vector<int> to(ss.leaves.size(), -1);
      std::vector<char> used(sp.size(), 0);
      bool ok = true;
      for (size_t l = 0; l < ss.leaves.size() && ok; ++l) {
        for (size_t k = 0; k < sp.size(); ++k)
          if (!used[k] && same(ss.leaves[l], sp[k])) {
            to[l] = (int)k;
            used[k] = 1;
            break;
          }
        ok = to[l] >= 0;
      }
      if (!ok) continue;
      plan.push_back({t, to});
      words += ss.leaves.size() * (size_t)((dsegs[ss.dseg].num_docs + 63) / 64);
    }
    if (!plan.empty()) {
      unsigned long long* buf = scratch.alloc<unsigned long long>(words);
      size_t off = 0;
      for (auto& pl_ : plan) {
        StatSeg& ss = stat_segs[pl_.first];
        DevSegment& d = dsegs[ss.dseg];
        const size_t nw = (size_t)((d.num_docs + 63) / 64);
        ss.fused = buf + off;
        for (size_t l = 0; l < ss.leaves.size(); ++l)
          d.sp_lbits[pl_.second[l]] = reinterpret_cast<uint32_t*>(buf + off + l * nw);
        off += ss.leaves.size() * nw;
      }
    }
  }
  // the optimistic numGroupsLimit scan's segment table: no keep bitsets, no first-doc tables (copied after every
  // device pointer above is fixed up: r3 copied it before, so FK_CONJ set leaves scanned with null bitsets)
  std::vector<DevSegment> dsegs_opt;
  if (!limit_segs.empty() && limit_opt) {
    dsegs_opt = dsegs;
    for (auto& d : dsegs_opt) d.keep = nullptr, d.first_doc = nullptr;
  }

  check_interrupt();
  stamp("setup");
  if (!chunks.empty()) {
    DevSegment* d_segs = scratch.alloc<DevSegment>(dsegs.size());
    DevSegment* d_segs_opt = dsegs_opt.empty() ? nullptr : scratch.alloc<DevSegment>(dsegs_opt.size());
    FilterInsn* d_prog = scratch.alloc<FilterInsn>(std::max<size_t>(1, all_insns.size()));
    // the chunks + the numGroupsLimit pass's chunks (limit segments only; without them the list uploads as built)
    std::vector<Chunk> limit_chunks;
    for (int k : limit_segs)
      limit_chunks.insert(limit_chunks.end(), chunks.begin() + dseg_chunks[k].first, chunks.begin() + dseg_chunks[k].second);
    const size_t n_limit_chunks = limit_chunks.size();
    const size_t n_all_chunks = chunks.size() + n_limit_chunks;
    Chunk* d_chunks = scratch.alloc<Chunk>(n_all_chunks);
    const size_t b1 = sizeof(DevSegment) * dsegs.size(), b2 = sizeof(FilterInsn) * all_insns.size(),
                 b3 = sizeof(Chunk) * n_all_chunks, b4 = sizeof(DevSegment) * dsegs_opt.size();
    uint8_t* stage = static_cast<uint8_t*>(lane.lane->host_staging(b1 + b2 + b3 + b4));
    memcpy(stage, dsegs.data(), b1);
    memcpy(stage + b1, all_insns.data(), b2);
    if (!chunks.empty()) memcpy(stage + b1 + b2, chunks.data(), sizeof(Chunk) * chunks.size());
    if (n_limit_chunks) memcpy(stage + b1 + b2 + sizeof(Chunk) * chunks.size(), limit_chunks.data(), sizeof(Chunk) * n_limit_chunks);
    if (b4) memcpy(stage + b1 + b2 + b3, dsegs_opt.data(), b4);
    PH_HIP_CHECK(hipMemcpyAsync(d_segs, stage, b1, hipMemcpyHostToDevice, st));
    if (b2) PH_HIP_CHECK(hipMemcpyAsync(d_prog, stage + b1, b2, hipMemcpyHostToDevice, st));
    PH_HIP_CHECK(hipMemcpyAsync(d_chunks, stage + b1 + b2, b3, hipMemcpyHostToDevice, st));
    if (b4) PH_HIP_CHECK(hipMemcpyAsync(d_segs_opt, stage + b1 + b2 + b3, b4, hipMemcpyHostToDevice, st));
    PH_HIP_CHECK(hipEventRecord(lane.lane->ev_uploaded, st));  // the statistics pass (stream b) starts here
    stamp("uploaded");
    // container mode skipped the doc bitmaps; a numGroupsLimit first-seen pass runs the segments' generic programs,
    // which read them: build them then, patch the programs / segment tables and upload them again
    bool late_built = false;
    auto late_bitmaps = [&]() {
      if (!kp.group_cont || late_built) return;
      build_bitmaps();
      for (auto& bf : bitmap_fix) all_insns[bf.first].ptr = bitmap_dev[bf.second];
      for (auto* v : {&dsegs, &dsegs_opt}) {
        if (v->empty()) continue;
        for (auto& fb : fbitmap_fix) (*v)[fb.first].fptr = bitmap_dev[fb.second];
        for (auto& sb : sbm_fix) (*v)[sb.first / kSparseBitmaps].sp_bm[sb.first % kSparseBitmaps] = bitmap_dev[sb.second];
      }
      PH_HIP_CHECK(hipStreamSynchronize(st));  // nothing in flight reads the tables while they are replaced
      if (!all_insns.empty())
        copy_h2d_sync(d_prog, all_insns.data(), sizeof(FilterInsn) * all_insns.size());
      copy_h2d_sync(d_segs, dsegs.data(), sizeof(DevSegment) * dsegs.size());
      if (d_segs_opt)
        copy_h2d_sync(d_segs_opt, dsegs_opt.data(), sizeof(DevSegment) * dsegs_opt.size());
      late_built = true;
    };
    kp.segs = d_segs;
    kp.prog = d_prog;
    kp.chunks = d_chunks;
    kp.lds_bytes = (int32_t)lds;
    if (mode != MODE_PARTITION) {
      kp.chunk_begin = 0;
      kp.chunk_end = (int32_t)chunks.size();
      int blocks_per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / std::max<size_t>(lds, 1)));
      if (mode == MODE_GROUP_LDS) blocks_per_cu = std::min(blocks_per_cu, 4);
      if (kp.count_reg) blocks_per_cu = 4;  // 16 waves per CU, each with two tiles of loads in flight
      const int grid = (int)std::min<int64_t>((int64_t)chunks.size(), (int64_t)ctx->num_cus * blocks_per_cu);
      stats.scan_kernel = kp.count_reg  ? PH_KERNEL_COUNT_REG
                          : kp.agg_cont   ? PH_KERNEL_AGG_CONTAINERS
                          : kp.agg_sparse ? PH_KERNEL_AGG_SPARSE
                          : kp.agg_fast  ? PH_KERNEL_AGG_LEAN
                          : kp.group_cont ? PH_KERNEL_GROUP_CONTAINERS
                          : kp.group_sparse ? PH_KERNEL_GROUP_SPARSE
                          : kp.group_reg  ? PH_KERNEL_GROUP_REG
                          : kp.lds_fast  ? PH_KERNEL_GROUP_LDS_LEAN
                                         : PH_KERNEL_SCAN;
      // device_ms opens here: it covers the numGroupsLimit pass and (below) the bitmap build too
      PH_HIP_CHECK(hipEventRecord(lane.lane->ev_start, st));
      // an interruptible call scans in batches of kInterruptChunks chunks and checks between them
      const int32_t nchunks = (int32_t)chunks.size();
      int32_t step = interruptible ? kInterruptChunks : nchunks;
      if (ctx->has(OPT_INTERRUPT_CHUNKS) && interruptible) step = (int32_t)std::max<int64_t>(1, ctx->opt(OPT_INTERRUPT_CHUNKS));
      auto run_scan = [&](KParams kx) {
        for (int32_t cb = 0; cb < nchunks; cb += step) {
          kx.chunk_begin = cb;
          kx.chunk_end = std::min(nchunks, cb + step);
          launch_scan(kx, mode, q->num_group_by, 0, std::min(grid, kx.chunk_end - cb), lds, st);
          if (interruptible && kx.chunk_end < nchunks) {
            PH_HIP_CHECK(hipStreamSynchronize(st));
            check_interrupt();
          }
        }
      };
      bool scanned = false;
      if (!limit_segs.empty() && limit_opt) {
        KParams ko = kp;
        ko.segs = d_segs_opt;
        ko.late_prefetch = base_late;
        run_scan(ko);
        unsigned long long* keys_dev = scratch.alloc<unsigned long long>(1);
        launch_count_nonzero(kp.out_count, TR, keys_dev, st);
        PinnedBlock keys_host(ctx, st, 8);
        PH_HIP_CHECK(hipMemcpyAsync(keys_host.p, keys_dev, 8, hipMemcpyDeviceToHost, st));
        PH_HIP_CHECK(hipStreamSynchronize(st));
        const int64_t merged_keys = (int64_t)*keys_host.as<unsigned long long>();
        keys_host.release();
        if (merged_keys < group_limit) {
          scanned = true;  // no segment can hold `limit` keys: the untruncated scan is the reference's result
          stats.limit_pass = 1;
        } else if (mode == MODE_GROUP_HASH) {
          late_bitmaps();
          // truncation over a key space beyond the dense budget (LongMapBasedHolder / ArrayMapBasedHolder regime,
          // DictionaryBasedGroupKeyGenerator.java:629-637,809-817): the segments that cannot reach the limit are
          // rescanned in one launch; each limit segment then runs, one at a time, (1) a first-seen pass into its
          // own hash table (slot -> first matching doc of the slot's key), (2) the selection of the slots whose
          // keys are among the first `limit` (the dense path's k_limit_* kernels over slots instead of keys), and
          // (3) its scan, which looks each key's slot up in that table and aggregates only kept keys
          scanned = true;
          stats.limit_pass = 2;
          init_tables();
          PH_HIP_CHECK(hipMemsetAsync(kp.matched_total, 0, 8, st));
          if (kp.filter_entries) PH_HIP_CHECK(hipMemsetAsync(kp.filter_entries, 0, 8, st));
          std::vector<char> is_lim(dsegs.size(), 0);
          int32_t maxdocs = 1;
          for (int k : limit_segs) {
            is_lim[k] = 1;
            maxdocs = std::max(maxdocs, dsegs[k].num_docs);
          }
          int64_t H2 = 1024;
          while (H2 < 2 * (int64_t)maxdocs) H2 <<= 1;
          unsigned long long* hk2 = scratch.alloc<unsigned long long>((size_t)H2);
          uint32_t* first2 = scratch.alloc<uint32_t>((size_t)H2);
          uint32_t* keep2 = scratch.alloc<uint32_t>((size_t)(H2 + 31) / 32);
          const int64_t dbw = (int64_t)maxdocs / 32 + 2;
          uint32_t* docbits = scratch.alloc<uint32_t>((size_t)dbw);
          limit_scal = scratch.alloc<unsigned long long>(3 * limit_segs.size());
          PH_HIP_CHECK(hipMemsetAsync(limit_scal, 0, 24 * limit_segs.size(), st));
          // segment table of the limit rescans: every limit segment's keep bitset is keep2 (one segment at a time)
          std::vector<DevSegment> dl = dsegs_opt;
          for (int k : limit_segs) dl[k].keep = keep2;
          DevSegment* d_segs_lim = scratch.alloc<DevSegment>(dl.size());
          copy_h2d_sync(d_segs_lim, dl.data(), sizeof(DevSegment) * dl.size());
          auto launch_range = [&](KParams kx, int32_t cb, int32_t ce) {
            if (ce <= cb) return;
            kx.chunk_begin = cb;
            kx.chunk_end = ce;
            launch_scan(kx, mode, q->num_group_by, 0, std::min(grid, ce - cb), lds, st);
          };
          // the segments that cannot reach the limit: contiguous chunk ranges of non-limit segments
          {
            KParams kn = kp;
            kn.segs = d_segs_opt;
            kn.late_prefetch = base_late;
            int32_t cb = -1, ce = -1;
            for (size_t k = 0; k < dsegs.size(); ++k) {
              if (is_lim[k]) continue;
              if (dseg_chunks[k].first != ce) {
                launch_range(kn, cb, ce);
                cb = dseg_chunks[k].first;
              }
              ce = dseg_chunks[k].second;
            }
            launch_range(kn, cb, ce);
          }
          for (size_t t = 0; t < limit_segs.size(); ++t) {
            const int k = limit_segs[t];
            PH_HIP_CHECK(hipMemsetAsync(hk2, 0xFF, 8 * (size_t)H2, st));
            PH_HIP_CHECK(hipMemsetAsync(first2, 0xFF, 4 * (size_t)H2, st));
            PH_HIP_CHECK(hipMemsetAsync(docbits, 0, 4 * (size_t)dbw, st));
            KParams k1 = kp;  // (1) first-seen pass: no aggregation, no matched count
            k1.segs = d_segs_opt;
            k1.late_prefetch = 1;
            k1.matched_total = nullptr;
            k1.filter_entries = nullptr;
            k1.hkeys = hk2;
            k1.hmask = H2 - 1;
            k1.first_doc = first2;
            launch_range(k1, dseg_chunks[k].first, dseg_chunks[k].second);
            launch_limit_select(first2, H2, group_limit, 1, dbw, docbits, keep2, limit_scal + 3 * t, st);  // (2)
            KParams k2 = kp;  // (3) the truncated scan
            k2.segs = d_segs_lim;
            k2.late_prefetch = 1;
            k2.lkeys = hk2;
            k2.lmask = H2 - 1;
            launch_range(k2, dseg_chunks[k].first, dseg_chunks[k].second);
          }
        } else {
          init_tables();  // truncation needed: first-seen pass, then the rescan with keep bitsets
          PH_HIP_CHECK(hipMemsetAsync(kp.matched_total, 0, 8, st));
          if (kp.filter_entries) PH_HIP_CHECK(hipMemsetAsync(kp.filter_entries, 0, 8, st));
        }
      }
      if (!scanned && !limit_segs.empty()) {
        late_bitmaps();
        stats.limit_pass = 2;
        // first-seen pass over every limit segment in ONE launch (MODE_GROUP_GLOBAL records each key's first
        // matching doc in the segment's own table), then the kept keys of every segment in one select step; the
        // pass walks the limit segments' chunks, appended after the main chunk list
        int32_t maxdocs = 0;
        for (int k : limit_segs) maxdocs = std::max(maxdocs, dsegs[k].num_docs);
        const int64_t dbw = (int64_t)maxdocs / 32 + 2;
        uint32_t* docbits = scratch.alloc<uint32_t>((size_t)dbw * limit_segs.size());
        PH_HIP_CHECK(hipMemsetAsync(limit_first, 0xff, 4 * (size_t)G * limit_segs.size(), st));
        PH_HIP_CHECK(hipMemsetAsync(docbits, 0, 4 * (size_t)dbw * limit_segs.size(), st));
        KParams k1 = kp;
        k1.matched_total = nullptr;
        k1.filter_entries = nullptr;
        k1.late_prefetch = 1;
        k1.first_doc = limit_first;  // the pass flag; each segment writes its own table
        k1.gc_slots = 0;             // the pass aggregates nothing (and its LDS holds only the staging)
        k1.chunk_begin = (int32_t)chunks.size();
        k1.chunk_end = (int32_t)(chunks.size() + n_limit_chunks);
        const size_t lds1 = (size_t)kWaves * kp.stage_stride + 16;
        const int g1 = std::min<int>(k1.chunk_end - k1.chunk_begin, ctx->num_cus * 4);
        if (g1 > 0) launch_scan(k1, MODE_GROUP_GLOBAL, q->num_group_by, 0, g1, lds1, st);
        launch_limit_select(limit_first, G, group_limit, (int)limit_segs.size(), dbw, docbits, limit_keep, limit_scal,
                            st);
      }
      if (!scanned) run_scan(kp);
      PH_HIP_CHECK(hipEventRecord(lane.lane->ev_stop, st));
    } else {
      // ---- partitioned group-by: batches of chunks; kernel A (filter + decode + partition) on `st`,
      // kernel B (per-partition LDS aggregation + owned merge) on stream_b, overlapped across batches.
      // A batch's records (~batch_rows x selectivity x 4 B, double-buffered) stay resident in the 256 MiB
      // Infinity Cache between kernel A's writes and kernel B's reads.
      const bool has_sum = nvals && (val_ops[0] & 1), has_min = nvals && (val_ops[0] & 2),
                 has_max = nvals && (val_ops[0] & 4);
      int klo = kPartKeysLog2;
      if (ctx->has(OPT_PART_KLO)) klo = (int)std::max<int64_t>(8, std::min<int64_t>(13, ctx->opt(OPT_PART_KLO)));  // (13: kernel B table 128 KiB)
      while (klo > 8 && (G >> (klo - 1)) < 256) --klo;  // small key spaces: more partitions, more workgroups
      const int64_t P = (G + (int64_t(1) << klo) - 1) >> klo;
      if (P > kPartMaxParts) fail(PH_ERR_UNSUPPORTED, "partitioned group-by too large");
      const int vbits = nvals ? std::max(1, bits_for_range((uint64_t)(vmax - vmin))) : 0;
      rec64 = (klo + vbits > 32) ? 1 : 0;
      int64_t batch_rows = int64_t(1) << 31;  // one batch: launch tails of many short batches cost more than MALL reuse saves
      if (ctx->has(OPT_PART_BATCH_ROWS)) batch_rows = std::max<int64_t>(1 << 16, ctx->opt(OPT_PART_BATCH_ROWS));
      if (interruptible) batch_rows = std::min<int64_t>(batch_rows, (int64_t)kInterruptChunks * kChunkWords * 64);
      // batches: contiguous chunk ranges of ~batch_rows docs
      std::vector<std::pair<int32_t, int32_t>> batches;
      int64_t max_batch_docs = 0;
      if (chunk_docs_total < batch_rows) {  // one batch (config 3: no walk over its 61K chunks)
        batches.push_back({0, (int32_t)chunks.size()});
        max_batch_docs = chunk_docs_total;
      } else {
        int32_t b0 = 0;
        int64_t acc = 0;
        for (int32_t c = 0; c < (int32_t)chunks.size(); ++c) {
          acc += (int64_t)(chunks[c].word_end - chunks[c].word_begin) * 64;
          if (acc >= batch_rows || c + 1 == (int32_t)chunks.size()) {
            batches.push_back({b0, c + 1});
            max_batch_docs = std::max(max_batch_docs, acc);
            b0 = c + 1;
            acc = 0;
          }
        }
      }
      kp.part_klo = klo;
      // the next tile's loads go out before the flush (r2: 3.78 vs 4.39 ms on one box); PH_PART_FLUSH_FIRST
      // restores the r1 order
      kp.part_load_first = !ctx->has(OPT_PART_FLUSH_FIRST);
      kp.part_depth = 1;
      if (ctx->has(OPT_PART_DEPTH)) kp.part_depth = ctx->opt(OPT_PART_DEPTH) == 2 ? 2 : 1;
      // register-direct kernel A (k_part_reg): 32-bit records, <= 3 key columns, filter / key streams <= 16 bits
      // and a value stream <= 32 bits (the lane's dwords of a stream are one register window of 4 * CK / 4 * CV)
      kp.part_reg = 0;
      if (kp.part_fast && !rec64 && q->num_group_by <= 3 && !ctx->has(OPT_PART_LDS) && kp.part_depth == 1) {
        int kb = 1, vb = 1;
        for (auto& d : dsegs) {
          if (d.fkind == FK_RANGE) kb = std::max(kb, (int)d.streams[kp.f_stream].bits);
          for (int gi = 0; gi < q->num_group_by; ++gi) kb = std::max(kb, (int)d.streams[kp.g_stream[gi]].bits);
          if (nvals) vb = std::max(vb, (int)d.streams[kp.v_stream[0]].bits);
        }
        if (kb <= 16 && vb <= 32) {
          kp.part_reg = 1;
          kp.part_ck = (kb <= 12 && vb <= 20) ? 3 : 4;
          kp.part_cv = kp.part_ck == 3 ? 5 : 8;
          kp.stage_stride = 0;  // no staging
        }
      }
      stats.scan_kernel = !kp.part_fast ? PH_KERNEL_PART_SCAN
                          : kp.part_reg ? PH_KERNEL_PART_REG
                          : kp.part_depth == 2 ? PH_KERNEL_PART_LEAN2 : PH_KERNEL_PART_LEAN;
      // record = (key << vbits) | value offset, with vbits = 32 - klo in k_part_reg's form ((key << (32 - klo)) + value
      // offset: the shift itself drops the partition bits); the LDS-staged forms keep the key's low klo bits masked
      kp.part_vbits = kp.part_reg ? 32 - klo : vbits;
      kp.num_parts = (int32_t)P;
      kp.part_sets = 2;
      const int ring_log2 = ctx->has(OPT_PART_RING_LOG2) ? (int)ctx->opt(OPT_PART_RING_LOG2) : 5;
      size_t lds_a = partition_lds_bytes(kp, ring_log2);
      int a_cap = 4;  // 8-wave workgroups: <= 4 per CU (32 waves)
      if (kp.part_reg) {
        a_cap = part_reg_blocks_per_cu(kp, q->num_group_by, lds_a);  // 4-wave groups, VGPR-bound
        // one ring set only when two sets would leave a single workgroup per CU
        KParams k1 = kp;
        k1.part_sets = 1;
        const size_t lds1 = partition_lds_bytes(k1, ring_log2);
        const int cap1 = part_reg_blocks_per_cu(k1, q->num_group_by, lds1);
        const size_t per2 = std::min<size_t>(a_cap, (160 * 1024) / lds_a), per1 = std::min<size_t>(cap1, (160 * 1024) / lds1);
        int force = 0;
        if (ctx->has(OPT_PART_SETS)) force = (int)ctx->opt(OPT_PART_SETS);
        // r6 (config 3): two sets at 2 workgroups per CU 2.69-2.73 ms against one set at 3 per CU 2.71-2.76: two sets
        // unless they leave one workgroup per CU
        if (force == 1 || (force != 2 && per2 < 2 && per1 > per2)) {
          kp = k1;
          lds_a = lds1;
          a_cap = cap1;
        }
      }
      if (ctx->has(OPT_PART_WG_PER_CU)) a_cap = (int)std::max<int64_t>(1, std::min<int64_t>(8, ctx->opt(OPT_PART_WG_PER_CU)));
      const int a_per_cu = (int)std::max<size_t>(1, std::min<size_t>(a_cap, (160 * 1024) / lds_a));
      const int grid_a = ctx->num_cus * a_per_cu;
      int max_batch_chunks = 0;
      for (auto& bt : batches) max_batch_chunks = std::max(max_batch_chunks, bt.second - bt.first);
      // region (partition, workgroup) capacity: a workgroup scans <= ceil(chunks / grid) chunks; uniform keys
      // put 1/P of its docs in each partition; 25 % headroom + 64, rounded to 64 records (16-byte aligned
      // regions).  Skew beyond that spills to the overflow table.
      const int32_t max_chunk_words = std::max<int32_t>(1, chunk_words_max);
      const int64_t wg_docs = (int64_t)((max_batch_chunks + grid_a - 1) / grid_a) * max_chunk_words * 64;
      int64_t cap = (int64_t)((double)wg_docs * 1.25 / (double)P) + 64;
      cap = (cap + 63) / 64 * 64;
      // the ring word keeps flushed / chunk in 16 bits; ranks beyond the capacity go to the overflow table
      cap = std::min<int64_t>(cap, 65535 * (rec64 ? 8 : 16));
      const int64_t max_part_records = cap * grid_a;
      // COUNT and the value-offset SUM share one 64-bit LDS word in kernel B when both fit
      const bool pack_cs = !rec64 && max_part_records < (int64_t(1) << 24) &&
                           (vbits == 0 || (double)max_part_records * (double)((int64_t(1) << vbits) - 1) <
                                              (double)(int64_t(1) << 40));
      const size_t rec_bytes = rec64 ? 8 : 4;
      void* bufs[2];
      uint32_t* counts[2];
      for (int b = 0; b < 2; ++b) {
        if (b == 1 && batches.size() == 1) {  // one batch: no double buffering
          bufs[1] = bufs[0];
          counts[1] = counts[0];
          break;
        }
        bufs[b] = scratch.alloc<uint8_t>((size_t)P * grid_a * cap * rec_bytes);
        counts[b] = scratch.alloc<uint32_t>((size_t)P * grid_a);
      }
      stamp("part regions");
      kp.ovf_count = scratch.alloc<unsigned long long>(G);
      PH_HIP_CHECK(hipMemsetAsync(kp.ovf_count, 0, 8 * G, st));
      if (has_sum) {
        kp.ovf_sum = scratch.alloc<int64_t>(G);
        PH_HIP_CHECK(hipMemsetAsync(kp.ovf_sum, 0, 8 * G, st));
      }
      if (has_min) {
        kp.ovf_min = scratch.alloc<int64_t>(G);
        launch_fill_i64(kp.ovf_min, INT64_MAX, G, st);
      }
      if (has_max) {
        kp.ovf_max = scratch.alloc<int64_t>(G);
        launch_fill_i64(kp.ovf_max, INT64_MIN, G, st);
      }
      kp.part_cap = (int32_t)cap;
      // k_part_reg's fixed-count flush: thread t owns partition t, 32-slot rings, a workgroup's regions addressable
      // by one buffer descriptor
      kp.part_vbase = nvals ? vmin : 0;
      kp.lds_bytes = (int32_t)lds_a;
      PartAggParams bp{};
      bp.num_parts = (int32_t)P;
      bp.part_cap = (int32_t)cap;
      bp.part_klo = klo;
      bp.part_vbits = kp.part_vbits;
      bp.rec64 = rec64;
      bp.has_sum = has_sum;
      bp.has_min = has_min;
      bp.has_max = has_max;
      bp.pack_cs = pack_cs;
      bp.part_vbase = kp.part_vbase;
      bp.num_groups = G;
      bp.out_count = kp.out_count;
      bp.out_sum = has_sum ? reinterpret_cast<int64_t*>(kp.out_sum[0]) : nullptr;
      bp.out_min = has_min ? kp.out_min[0] : nullptr;
      bp.out_max = has_max ? kp.out_max[0] : nullptr;
      // kernel B slices: about one (partition, slice) workgroup per CU; a single slice owns its key range (no
      // device atomics in the merge).  r2 sweep, config 3 (P = 245): 1 slice 3.89, 2 slices 3.90, 3 slices 3.99 ms
      int slices = (int)std::max<int64_t>(1, std::min<int64_t>(8, (int64_t)ctx->num_cus / P));
      if (ctx->has(OPT_PART_SLICES)) slices = (int)std::max<int64_t>(1, std::min<int64_t>(16, ctx->opt(OPT_PART_SLICES)));
      bp.slices = slices;
      bp.mm_blind = ctx->has(OPT_PART_MM_BLIND) ? (int)ctx->opt(OPT_PART_MM_BLIND) : 0;
      bp.regions = grid_a;
      const size_t lds_b = part_agg_lds_bytes(bp);
      Lane& L = *lane.lane;
      // PH_PART_SERIAL=1 runs kernel B on the scan stream (profiling each kernel without overlap)
      hipStream_t sb = ctx->has(OPT_PART_SERIAL) ? st : L.stream_b;
      stamp("part fills");
      PH_HIP_CHECK(hipEventRecord(L.ev_start, st));
      for (size_t b = 0; b < batches.size(); ++b) {
        if (interruptible && b > 0) {
          PH_HIP_CHECK(hipStreamSynchronize(st));
          PH_HIP_CHECK(hipStreamSynchronize(sb));
          check_interrupt();
        }
        const int set = (int)(b & 1);
        if (b >= 2) PH_HIP_CHECK(hipStreamWaitEvent(st, L.event(2 * (b - 2) + 1), 0));  // set free again
        kp.chunk_begin = batches[b].first;
        kp.chunk_end = batches[b].second;
        kp.part_buf = bufs[set];
        kp.part_count = counts[set];
        const int nch = kp.chunk_end - kp.chunk_begin;
        const int grid = std::min(nch, grid_a);
        launch_scan(kp, MODE_PARTITION, q->num_group_by, rec64, grid, lds_a, st);
        PH_HIP_CHECK(hipEventRecord(L.event(2 * b), st));
        PH_HIP_CHECK(hipStreamWaitEvent(sb, L.event(2 * b), 0));
        bp.part_buf = bufs[set];
        bp.part_count = counts[set];
        bp.regions = grid;
        launch_part_agg(bp, lds_b, sb);
        PH_HIP_CHECK(hipEventRecord(L.event(2 * b + 1), sb));
      }
      MergeParams mp{kp.out_count, bp.out_sum, bp.out_min, bp.out_max, kp.ovf_count, kp.ovf_sum, kp.ovf_min,
                     kp.ovf_max, G};
      PH_HIP_CHECK(hipEventRecord(L.event(2 * batches.size()), st));
      PH_HIP_CHECK(hipStreamWaitEvent(sb, L.event(2 * batches.size()), 0));
      launch_merge_overflow(mp, sb);
      PH_HIP_CHECK(hipEventRecord(L.event(2 * batches.size() + 1), sb));
      PH_HIP_CHECK(hipStreamWaitEvent(st, L.event(2 * batches.size() + 1), 0));
      PH_HIP_CHECK(hipEventRecord(L.ev_stop, st));
    }
    // numEntriesScannedInFilter of the ST_SCANAND / ST_SIM segments (a statistics pass on the second stream, after
    // the scan's device-time window and overlapping its kernels: it reads only the forward indexes): the leaves' doc
    // bitmaps (k_leaf_bitmaps from the forward indexes, k_filter_bitmaps for the rest), then
    // the chunked walks of the AND-of-scans leap-frog on the device (k_and_walk) or the iterator simulation on the
    // host, in batches of segments bounded to kStatBatchWords words of bitmaps
    if (!stat_segs.empty()) {
      hipStream_t sb = lane.lane->stream_b;
      PH_HIP_CHECK(hipStreamWaitEvent(sb, lane.lane->ev_uploaded, 0));
      constexpr size_t kStatBatchWords = (size_t)32 << 20;  // 256 MiB
      auto seg_words = [&](const StatSeg& ss) {
        return ss.leaves.size() * (size_t)((dsegs[ss.dseg].num_docs + 63) / 64);
      };
      size_t total = 0, biggest = 0, n_scanand = 0, walk_tab = 0;
      int32_t walk_k = 2;
      for (auto& ss : stat_segs)
        if (ss.dseg >= 0 && ss.kind == ST_SCANAND) walk_k = std::max(walk_k, (int32_t)ss.leaves.size());
      const int dfa_block = and_dfa_block(walk_k);
      auto walk_groups = [&](int64_t n) {
        const int64_t nch = (n + and_dfa_chunk_words() * 64 - 1) / (and_dfa_chunk_words() * 64);
        return (nch + dfa_block - 1) / dfa_block;
      };
      for (auto& ss : stat_segs) {
        if (ss.dseg < 0) continue;
        if (!ss.fused) {  // a fused AND's bitmaps are the scan's (no batch buffer)
          total += seg_words(ss);
          biggest = std::max(biggest, seg_words(ss));
        }
        n_scanand += ss.kind == ST_SCANAND;
        if (ss.kind == ST_SCANAND)
          walk_tab += (size_t)(ss.leaves.size() + 1) * (size_t)walk_groups(dsegs[ss.dseg].num_docs);
      }
      const size_t cap_words = std::max<size_t>(1, std::min(total, std::max(kStatBatchWords, biggest)));
      unsigned long long* dev = scratch.alloc<unsigned long long>(cap_words);
      // the walks' workgroup tables ((k + 1) x groups per AND)
      uint32_t* d_wdelta = walk_tab ? scratch.alloc<uint32_t>(walk_tab) : nullptr;
      uint8_t* d_wexit = walk_tab ? scratch.alloc<uint8_t>(walk_tab) : nullptr;
      AndWalkJob* d_wjobs = n_scanand ? scratch.alloc<AndWalkJob>(n_scanand) : nullptr;
      unsigned long long* d_out = n_scanand ? scratch.alloc<unsigned long long>(n_scanand) : nullptr;
      size_t n_fast = 0, set_words = 0;
      for (auto& ss : stat_segs)
        for (auto& l : ss.leaves)
          if (ss.dseg >= 0 && fast_leaf(l)) {
            ++n_fast;
            set_words += l.op == OP_SET ? l.set.size() : 0;
          }
      LeafJob* d_ljobs = n_fast ? scratch.alloc<LeafJob>(n_fast) : nullptr;
      uint32_t* d_lsets = set_words ? scratch.alloc<uint32_t>(set_words) : nullptr;
      std::vector<int64_t> ent(stat_segs.size(), 0);
      size_t tab_used = 0;  // walk tables handed out so far (fused ANDs first, then the batches')
      // the fused ANDs' walks: after the scan that wrote their leaf bitmaps (ev_stop on the scan stream)
      {
        std::vector<AndWalkJob> wj;
        std::vector<size_t> who;
        int64_t max_groups = 0;
        int32_t max_k = 0;
        for (size_t t = 0; t < stat_segs.size(); ++t) {
          const StatSeg& ss = stat_segs[t];
          if (!ss.fused || ss.dseg < 0) continue;
          const int64_t n = dsegs[ss.dseg].num_docs;
          AndWalkJob J{};
          J.bits = ss.fused;
          J.nwords = (n + 63) / 64;
          J.ndocs = n;
          J.k = (int32_t)ss.leaves.size();
          J.slot = (int32_t)wj.size();
          J.nchunks = (n + and_dfa_chunk_words() * 64 - 1) / (and_dfa_chunk_words() * 64);
          J.ngroups = (int32_t)walk_groups(n);
          J.gdelta = d_wdelta + tab_used;
          J.gexit = d_wexit + tab_used;
          tab_used += (size_t)(J.k + 1) * (size_t)J.ngroups;
          max_groups = std::max<int64_t>(max_groups, J.ngroups);
          max_k = std::max(max_k, J.k);
          wj.push_back(J);
          who.push_back(t);
        }
        if (!wj.empty()) {
          PH_HIP_CHECK(hipStreamWaitEvent(sb, lane.lane->ev_stop, 0));
          PH_HIP_CHECK(hipMemcpyAsync(d_wjobs, wj.data(), sizeof(AndWalkJob) * wj.size(), hipMemcpyHostToDevice, sb));
          launch_and_walk(d_wjobs, (int32_t)wj.size(), max_groups, max_k, d_out, sb);
          fused_blk = std::make_unique<PinnedBlock>(ctx, sb, 8 * wj.size());
          PH_HIP_CHECK(hipMemcpyAsync(fused_blk->p, d_out, 8 * wj.size(), hipMemcpyDeviceToHost, sb));
          fused_docs.clear();  // summed by finish_fused() at the end of the call
          for (size_t t : who) fused_docs.push_back(dsegs[stat_segs[t].dseg].num_docs);
        }
      }
      size_t next = 0;
      while (next < stat_segs.size()) {
        // the batch: whole segments up to cap_words words of bitmaps
        std::vector<size_t> batch, base;
        size_t used = 0;
        for (; next < stat_segs.size(); ++next) {
          const StatSeg& ss = stat_segs[next];
          if (ss.dseg < 0 || ss.fused) continue;
          if (!batch.empty() && used + seg_words(ss) > cap_words) break;
          batch.push_back(next);
          base.push_back(used);
          used += seg_words(ss);
        }
        if (batch.empty()) break;
        // leaf bitmaps: one k_leaf_bitmaps launch for the batch's forward-index leaves
        std::vector<LeafJob> lj;
        std::vector<uint32_t> lsets;
        int64_t max_docs = 0;
        int32_t max_bits = 1;
        for (size_t b = 0; b < batch.size(); ++b) {
          const StatSeg& ss = stat_segs[batch[b]];
          const int64_t n = dsegs[ss.dseg].num_docs, nw = (n + 63) / 64;
          ph_segment* sg = segs[ss.qi];
          for (size_t l = 0; l < ss.leaves.size(); ++l) {
            const PNode& lf = ss.leaves[l];
            if (!fast_leaf(lf)) continue;
            const Column* col = sg->columns.at(slot_names[lf.col]).get();
            LeafJob J{};
            J.fwd = (const uint32_t*)col->d_fwd.ptr;
            J.ndocs = n;
            J.bits = col->bits;
            J.lo = lf.op == OP_RANGE ? lf.lo : 0u;  // a set leaf matches through its bitset only (an empty one: none)
            J.len = lf.op == OP_RANGE ? lf.len : 0u;
            if (lf.op == OP_SET && !lf.set.empty()) {
              J.set = d_lsets + lsets.size();
              J.set_words = (int32_t)lf.set.size();
              J.card = (int32_t)std::min<int64_t>(col->cardinality, (int64_t)lf.set.size() * 32);
              lsets.insert(lsets.end(), lf.set.begin(), lf.set.end());
            }
            J.out = (uint32_t*)(dev + base[b] + l * (size_t)nw);
            J.out_words = 2 * nw;
            if (!J.fwd) fail(PH_ERR_DEVICE, "scan leaf without a forward index");
            lj.push_back(J);
            max_docs = std::max(max_docs, n);
            max_bits = std::max(max_bits, J.bits);
          }
          for (size_t j = 0; j < ss.jobs.size(); ++j) {
            FbJob job = fb_jobs[ss.jobs[j]];
            job.out = dev + base[b];
            launch_filter_bitmaps(d_prog, d_segs, job, sb);
          }
        }
        if (!lj.empty()) {
          if (!lsets.empty())
            PH_HIP_CHECK(hipMemcpyAsync(d_lsets, lsets.data(), 4 * lsets.size(), hipMemcpyHostToDevice, sb));
          // one launch per load-width class (1, 2, 4 or 8 16-byte loads per lane), jobs grouped by class
          auto cls = [](int32_t b) { return b <= 4 ? 0 : b <= 8 ? 1 : b <= 16 ? 2 : 3; };
          std::stable_sort(lj.begin(), lj.end(), [&](const LeafJob& a, const LeafJob& b) { return cls(a.bits) < cls(b.bits); });
          PH_HIP_CHECK(hipMemcpyAsync(d_ljobs, lj.data(), sizeof(LeafJob) * lj.size(), hipMemcpyHostToDevice, sb));
          for (size_t i = 0; i < lj.size();) {
            size_t e = i;
            int64_t nd = 0;
            int32_t mb = 1, sw = 0;
            while (e < lj.size() && cls(lj[e].bits) == cls(lj[i].bits)) {
              nd = std::max(nd, lj[e].ndocs);
              mb = std::max(mb, lj[e].bits);
              if (lj[e].set) sw = std::max(sw, lj[e].set_words);
              ++e;
            }
            launch_leaf_bitmaps(d_ljobs + i, (int32_t)(e - i), nd, mb, sw, sb);
            i = e;
          }
          (void)max_docs;
          (void)max_bits;
        }
        // the AND-of-scans walks: per-chunk transition tables composed per job (exact, one pass)
        std::vector<size_t> walk_b;  // batch positions of the scan-AND segments
        for (size_t b = 0; b < batch.size(); ++b)
          if (stat_segs[batch[b]].kind == ST_SCANAND) walk_b.push_back(b);
        std::vector<unsigned long long> out(walk_b.size(), 0);
        // the simulated segments' bitmaps go to the host (only theirs: the buffer is not touched otherwise)
        std::vector<size_t> hbase(batch.size(), 0);
        size_t hwords = 0;
        for (size_t b = 0; b < batch.size(); ++b)
          if (stat_segs[batch[b]].kind == ST_SIM) {
            hbase[b] = hwords;
            hwords += seg_words(stat_segs[batch[b]]);
          }
        std::unique_ptr<uint64_t[]> h(hwords ? new uint64_t[hwords] : nullptr);
        for (size_t b = 0; b < batch.size(); ++b)
          if (stat_segs[batch[b]].kind == ST_SIM)
            PH_HIP_CHECK(hipMemcpyAsync(h.get() + hbase[b], dev + base[b], 8 * seg_words(stat_segs[batch[b]]),
                                        hipMemcpyDeviceToHost, sb));
        if (!walk_b.empty()) {
          std::vector<AndWalkJob> wj;
          size_t tab = 0;
          int64_t max_groups = 0;
          int32_t max_k = 0;
          for (size_t t = 0; t < walk_b.size(); ++t) {
            const StatSeg& ss = stat_segs[batch[walk_b[t]]];
            const int64_t n = dsegs[ss.dseg].num_docs;
            AndWalkJob J{};
            J.bits = dev + base[walk_b[t]];
            J.nwords = (n + 63) / 64;
            J.ndocs = n;
            J.k = (int32_t)ss.leaves.size();
            J.slot = (int32_t)wj.size();
            J.nchunks = (n + and_dfa_chunk_words() * 64 - 1) / (and_dfa_chunk_words() * 64);
            J.ngroups = (int32_t)walk_groups(n);
            J.gdelta = d_wdelta + tab_used + tab;
            J.gexit = d_wexit + tab_used + tab;
            tab += (size_t)(J.k + 1) * (size_t)J.ngroups;
            max_groups = std::max<int64_t>(max_groups, J.ngroups);
            max_k = std::max(max_k, J.k);
            if (J.k < 2) fail(PH_ERR_DEVICE, "AND of fewer than two scans");
            wj.push_back(J);
          }
          PH_HIP_CHECK(hipMemcpyAsync(d_wjobs, wj.data(), sizeof(AndWalkJob) * wj.size(), hipMemcpyHostToDevice, sb));
          launch_and_walk(d_wjobs, (int32_t)wj.size(), max_groups, max_k, d_out, sb);
          PH_HIP_CHECK(hipMemcpyAsync(out.data(), d_out, 8 * wj.size(), hipMemcpyDeviceToHost, sb));
        }
        PH_HIP_CHECK(hipStreamSynchronize(sb));
        stamp("stat walk");
        for (size_t t = 0; t < walk_b.size(); ++t) {
          const StatSeg& ss = stat_segs[batch[walk_b[t]]];
          ent[batch[walk_b[t]]] = dsegs[ss.dseg].num_docs - 1 + (int64_t)out[t];
        }
        stamp("stat walks");
        // host simulations (ST_SIM segments), on a small pool; an exception in a worker is rethrown after the join
        std::vector<size_t> work_items;
        for (size_t b = 0; b < batch.size(); ++b)
          if (stat_segs[batch[b]].kind == ST_SIM) work_items.push_back(b);
        pool_run(work_items.size(), std::min(8u, std::max(1u, std::thread::hardware_concurrency())), [&](size_t t) {
          const size_t b = work_items[t];
          const StatSeg& ss = stat_segs[batch[b]];
          const int64_t n = dsegs[ss.dseg].num_docs, nw = (n + 63) / 64;
          std::vector<SimLeaf> lv(ss.leaves.size());
          for (size_t l = 0; l < lv.size(); ++l) lv[l] = {ss.leaf_kinds[l], h.get() + hbase[b] + l * (size_t)nw};
          ent[batch[b]] = simulate_filter_entries(ss.root, lv, n);
        });
      }
      for (int64_t e : ent) stats.num_entries_scanned_in_filter += e;
      stamp("stat pass");
    }
    stamp("launched");
    timed = true;
    if (!defer_sync) {
      PH_HIP_CHECK(hipStreamSynchronize(st));  // staging buffer reuse + results
      stamp("kernels done");
      dev_ms = device_elapsed();
    }
  } else {
    PH_HIP_CHECK(hipStreamSynchronize(st));
    dev_ms = device_elapsed();  // the bitmap build alone (no chunk to scan)
  }
  stats.device_ms = dev_ms;
  res->mode = mode;
  stats.plan_mode = mode;
  // words read back with the results: [0] matched docs, [1] applyAnd filter entries, [2..] 3 per limit segment
  if (kp.matched_total && defer_sync) {
    dsc_nlim = limit_scal ? limit_segs.size() : 0;
    dsc = std::make_unique<PinnedBlock>(ctx, st, 8 * (2 + 3 * dsc_nlim));
    unsigned long long* dw = dsc->as<unsigned long long>();
    dw[1] = 0;
    PH_HIP_CHECK(hipMemcpyAsync(dw, kp.matched_total, 8, hipMemcpyDeviceToHost, st));
    if (kp.filter_entries) PH_HIP_CHECK(hipMemcpyAsync(dw + 1, kp.filter_entries, 8, hipMemcpyDeviceToHost, st));
    if (dsc_nlim) PH_HIP_CHECK(hipMemcpyAsync(dw + 2, limit_scal, 24 * dsc_nlim, hipMemcpyDeviceToHost, st));
  } else if (kp.matched_total) {
    // group-by: numDocsScanned = matched docs (docs of keys beyond numGroupsLimit included,
    // GroupByOperator.java:106-107) and numGroupsLimitReached of any segment
    const size_t nlim = limit_scal ? limit_segs.size() : 0;
    std::vector<unsigned long long> sc(2 + 3 * nlim, 0);
    PH_HIP_CHECK(hipMemcpyAsync(sc.data(), kp.matched_total, 8, hipMemcpyDeviceToHost, st));
    if (kp.filter_entries) PH_HIP_CHECK(hipMemcpyAsync(sc.data() + 1, kp.filter_entries, 8, hipMemcpyDeviceToHost, st));
    if (nlim) PH_HIP_CHECK(hipMemcpyAsync(sc.data() + 2, limit_scal, 24 * nlim, hipMemcpyDeviceToHost, st));
    PH_HIP_CHECK(hipStreamSynchronize(st));
    stats.num_docs_scanned = (int64_t)sc[0];
    stats.num_entries_scanned_in_filter += (int64_t)sc[1];
    for (size_t t = 0; t < nlim; ++t) stats.num_groups_limit_reached |= sc[2 + 3 * t + 2] != 0;
  } else if (kp.filter_entries) {  // aggregation-only
    unsigned long long fe = 0;
    PH_HIP_CHECK(hipMemcpyAsync(&fe, kp.filter_entries, 8, hipMemcpyDeviceToHost, st));
    PH_HIP_CHECK(hipStreamSynchronize(st));
    stats.num_entries_scanned_in_filter += (int64_t)fe;
  }
  if (dop == DENSE_EXECUTE) {
    finish_fused();
    // partial tables stay on the device for the cross-GPU reduction
    stats.num_entries_scanned_post_filter = stats.num_docs_scanned * (int64_t)projected.size();
    stats.host_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count() - dev_ms;
    return res.release();
  }
  }  // !fin

  // ---- results (DENSE_FINALIZE: only the key shard [RB, RB + RG) of the tables)
  const int64_t RB = fin ? dn->g0 : 0;
  const int64_t RG = fin ? dn->g1 - dn->g0 : TR;
  const int64_t rhll_words = RG * num_hll * (m ? m : 1);
  const int ncols_proj = (int)projected.size();
  auto finish_value = [&](int k, int64_t raw, int64_t cnt_for_default, bool is_sum) -> double {
    const int j = agg_val[k];
    const int t = q->aggregations[k].type;
    double v;
    if (is_sum) {
      if (val_is_int[j]) {
        v = (double)raw;
        if (raw >= (int64_t(1) << 53) || raw <= -(int64_t(1) << 53)) stats.sum_precision_flag = 1;
      } else {
        memcpy(&v, &raw, 8);
      }
    } else if (cnt_for_default == 0) {
      v = t == PH_AGG_MIN ? INFINITY : -INFINITY;  // Min/MaxAggregationFunction defaults
    } else {
      v = val_is_int[j] ? (double)raw : double_from_order_key(raw);
    }
    return v;
  };
  auto src_of = [&](int k) -> void* {
    const int j = agg_val[k];
    const int t = q->aggregations[k].type;
    return t == PH_AGG_SUM ? kp.out_sum[j] : (t == PH_AGG_MIN ? (void*)kp.out_min[j] : (void*)kp.out_max[j]);
  };
  // after the first sync of the result path: the deferred scan timing and group-by statistics
  auto resolve_deferred = [&]() {
    if (defer_sync && timed) {
      stamp("kernels done");
      dev_ms = device_elapsed();
      stats.device_ms = dev_ms;
    }
    if (dsc) {
      const unsigned long long* dw = dsc->as<unsigned long long>();
      stats.num_docs_scanned = (int64_t)dw[0];
      stats.num_entries_scanned_in_filter += (int64_t)dw[1];
      for (size_t t = 0; t < dsc_nlim; ++t) stats.num_groups_limit_reached |= dw[2 + 3 * t + 2] != 0;
      dsc.reset();
    }
  };
  if (q->num_group_by == 0) {
    init_row_results(1);
    // every scalar (and HLL register block) in one round trip: async copies into one pinned block, one sync
    std::vector<size_t> at(nagg + 1, 0);
    size_t need = 8;
    for (int k = 0; k < nagg; ++k) {
      at[k] = need;
      const int t = q->aggregations[k].type;
      need += t == PH_AGG_COUNT ? 0 : (t == PH_AGG_DISTINCTCOUNTHLL ? 4 * (size_t)m : 8);
    }
    PinnedBlock blk_hold(ctx, st, need);
    uint8_t* blk = blk_hold.as<uint8_t>();
    PH_HIP_CHECK(hipMemcpyAsync(blk, kp.out_count, 8, hipMemcpyDeviceToHost, st));
    for (int k = 0; k < nagg; ++k) {
      const int t = q->aggregations[k].type;
      if (t == PH_AGG_DISTINCTCOUNTHLL)
        PH_HIP_CHECK(hipMemcpyAsync(blk + at[k], kp.out_hll + (size_t)agg_hll[k] * m, 4 * m, hipMemcpyDeviceToHost, st));
      else if (t != PH_AGG_COUNT)
        PH_HIP_CHECK(hipMemcpyAsync(blk + at[k], src_of(k), 8, hipMemcpyDeviceToHost, st));
    }
    PH_HIP_CHECK(hipStreamSynchronize(st));
    resolve_deferred();
    unsigned long long matched = 0;
    memcpy(&matched, blk, 8);
    stats.num_docs_scanned = (int64_t)matched;
    for (int k = 0; k < nagg; ++k) {
      const int t = q->aggregations[k].type;
      uint8_t* dst = res->aggs[k].data();
      if (t == PH_AGG_COUNT) {
        int64_t v = (int64_t)matched;
        memcpy(dst, &v, 8);
      } else if (t == PH_AGG_DISTINCTCOUNTHLL) {
        const uint32_t* r = reinterpret_cast<const uint32_t*>(blk + at[k]);
        for (int j = 0; j < m; ++j) dst[j] = (uint8_t)r[j];
      } else {
        int64_t raw;
        memcpy(&raw, blk + at[k], 8);
        double v = finish_value(k, raw, (int64_t)matched, t == PH_AGG_SUM);
        memcpy(dst, &v, 8);
      }
    }

  } else if (num_hll == 0) {
    // device-side compaction: non-empty groups in key order, keys decoded, values converted to double,
    // copied straight into pinned result columns
    CompactParams cp{};
    cp.num_groups = RG;
    cp.chunk = std::max<int64_t>(1024, (RG + kCompactBlocks - 1) / kCompactBlocks);
    cp.count = kp.out_count;
    cp.num_aggs = nagg;
    cp.num_keys = q->num_group_by;
    for (int k = 0; k < nagg; ++k) {
      const int t = q->aggregations[k].type;
      if (t == PH_AGG_COUNT) {
        cp.agg_kind[k] = CK_COUNT;
        continue;
      }
      const int j = agg_val[k];
      cp.agg_kind[k] = val_is_int[j] ? CK_INT : (t == PH_AGG_SUM ? CK_REAL_SUM : CK_REAL_ORDER);
      cp.agg_src[k] = reinterpret_cast<const int64_t*>(src_of(k));
      cp.agg_out[k] = scratch.alloc<double>(RG);
    }
    std::vector<int32_t> key_es(q->num_group_by);
    for (int g = 0; g < q->num_group_by; ++g) {
      GlobalDict& gd = *gdicts[g];
      cp.key_stride[g] = kp.group_stride[g];
      cp.key_size[g] = std::max<int64_t>(1, gd.dict.size);
      cp.key_type[g] = gd.dict.type;
      cp.key_table[g] = global_dict_device_values(ctx, gd);
      key_es[g] = (gd.dict.type == PH_LONG || gd.dict.type == PH_DOUBLE) ? 8 : 4;
      cp.key_out[g] = scratch.alloc<uint8_t>((size_t)RG * key_es[g]);
    }
    cp.count_out = scratch.alloc<int64_t>(RG);
    cp.key_base = RB;
    cp.hkeys = hkeys;
    cp.blk = scratch.alloc<unsigned long long>(kCompactBlocks + 2);
    PH_HIP_CHECK(hipMemsetAsync(cp.blk + kCompactBlocks + 1, 0, 8, st));
    launch_compact(cp, st);
    PinnedBlock tot_hold(ctx, st, 16);
    unsigned long long* tot = tot_hold.as<unsigned long long>();
    PH_HIP_CHECK(hipMemcpyAsync(tot, cp.blk + kCompactBlocks, 16, hipMemcpyDeviceToHost, st));
    PH_HIP_CHECK(hipStreamSynchronize(st));
    resolve_deferred();
    const int64_t R = (int64_t)tot[0];
    const int64_t docs = (int64_t)tot[1];
    tot_hold.release();
    res->num_groups = R;
    res->ctx = ctx;
    res->aggs.resize(nagg);
    // the columns' copies alternate between the two streams of the lane (two copy queues over PCIe) unless the fused
    // statistic walk still runs on the second one
    const bool two = !fused_blk;
    bool used_b = false;
    int cix = 0;
    auto take = [&](ResultBuf& b, const void* dsrc, size_t bytes) {
      b.pinned = ctx->pinned_acquire(bytes, &b.cap);
      b.n = bytes;
      if (!bytes) return;
      const bool on_b = two && (cix++ & 1);
      used_b |= on_b;
      PH_HIP_CHECK(hipMemcpyAsync(b.pinned, dsrc, bytes, hipMemcpyDeviceToHost, on_b ? lane.lane->stream_b : st));
    };
    for (int k = 0; k < nagg; ++k) {
      if (cp.agg_kind[k] == CK_COUNT) take(res->aggs[k], cp.count_out, 8 * (size_t)R);
      else take(res->aggs[k], cp.agg_out[k], 8 * (size_t)R);
    }

    res->key_types.resize(q->num_group_by);
    res->key_entry_size.resize(q->num_group_by);
    res->keys.resize(q->num_group_by);
    std::vector<ResultBuf> string_ids(q->num_group_by);
    struct IdsGuard {  // STRING keys' id columns: pinned blocks returned on every exit (a throw drains the stream)
      Context* c;
      hipStream_t s;
      std::vector<ResultBuf>& v;
      ~IdsGuard() {
        for (auto& b : v)
          if (b.pinned) {
            if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(s);
            c->pinned_release(b.pinned, b.cap);
            b.pinned = nullptr;
          }
      }
    } ids_guard{ctx, st, string_ids};
    for (int g = 0; g < q->num_group_by; ++g) {
      const Dictionary& d = gdicts[g]->dict;
      res->key_types[g] = d.type;
      if (d.type == PH_STRING) {
        take(string_ids[g], cp.key_out[g], 4 * (size_t)R);
      } else {
        res->key_entry_size[g] = key_es[g];
        take(res->keys[g], cp.key_out[g], (size_t)key_es[g] * R);
      }
    }
    PH_HIP_CHECK(hipStreamSynchronize(st));
    if (used_b) PH_HIP_CHECK(hipStreamSynchronize(lane.lane->stream_b));
    // a finalised key shard has no scan: its matched docs are the sum of its group counts (k_compact_count)
    if (fin) stats.num_docs_scanned = docs;
    for (int k = 0; k < nagg; ++k) {
      if (q->aggregations[k].type != PH_AGG_SUM || !val_is_int[agg_val[k]]) continue;
      if (!fin && sum_bounded[agg_val[k]]) continue;
      const double* sv = reinterpret_cast<const double*>(res->aggs[k].data());
      for (int64_t r = 0; r < R; ++r)
        if (sv[r] >= 9007199254740992.0 || sv[r] <= -9007199254740992.0) {
          stats.sum_precision_flag = 1;
          break;
        }
    }
    for (int g = 0; g < q->num_group_by; ++g) {
      if (res->key_types[g] != PH_STRING) continue;
      const Dictionary& d = gdicts[g]->dict;
      const int32_t es = key_entry_size(d);
      res->key_entry_size[g] = es;
      res->keys[g].assign((size_t)es * R, 0);
      const int32_t* ids = reinterpret_cast<const int32_t*>(string_ids[g].data());
      for (int64_t r = 0; r < R; ++r) put_key_value(d, ids[r], res->keys[g].data() + (size_t)es * r, es);
      ctx->pinned_release(string_ids[g].pinned, string_ids[g].cap);
      string_ids[g].pinned = nullptr;
    }
  } else {
    // group-by with DISTINCTCOUNTHLL registers: host-side materialisation (MODE_GROUP_HASH: rows are the occupied
    // slots, ordered by their raw key like the dense tables' rows)
    std::vector<unsigned long long> cnt(RG);
    PH_HIP_CHECK(hipMemcpy(cnt.data(), kp.out_count, 8 * RG, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> slot_key;
    if (mode == MODE_GROUP_HASH) {
      slot_key.resize(RG);
      PH_HIP_CHECK(hipMemcpy(slot_key.data(), hkeys, 8 * RG, hipMemcpyDeviceToHost));
    }
    std::vector<int64_t> live;
    int64_t docs = 0;
    for (int64_t g = 0; g < RG; ++g)
      if (cnt[g]) {
        live.push_back(g);
        docs += (int64_t)cnt[g];
      }
    if (!slot_key.empty())
      std::sort(live.begin(), live.end(), [&](int64_t a, int64_t b) { return slot_key[a] < slot_key[b]; });
    auto key_of = [&](int64_t row) -> int64_t { return slot_key.empty() ? RB + live[row] : (int64_t)slot_key[live[row]]; };
    if (fin) stats.num_docs_scanned = docs;
    const int64_t R = (int64_t)live.size();
    res->num_groups = R;
    init_row_results(R);
    std::map<void*, std::vector<int64_t>> fetched;
    std::vector<uint32_t> regs;
    for (int k = 0; k < nagg; ++k) {
      const int t = q->aggregations[k].type;
      uint8_t* dst = res->aggs[k].data();
      if (t == PH_AGG_COUNT) {
        for (int64_t r = 0; r < R; ++r) {
          int64_t v = (int64_t)cnt[live[r]];
          memcpy(dst + 8 * r, &v, 8);
        }
      } else if (t == PH_AGG_DISTINCTCOUNTHLL) {
        if (regs.empty()) {
          regs.resize(rhll_words);
          PH_HIP_CHECK(hipMemcpy(regs.data(), kp.out_hll, 4 * rhll_words, hipMemcpyDeviceToHost));
        }
        for (int64_t r = 0; r < R; ++r)
          for (int j = 0; j < m; ++j)
            dst[(size_t)r * m + j] = (uint8_t)regs[((size_t)live[r] * num_hll + agg_hll[k]) * m + j];
      } else {
        void* src = src_of(k);
        auto& buf = fetched[src];
        if (buf.empty()) {
          buf.resize(RG);
          PH_HIP_CHECK(hipMemcpy(buf.data(), src, 8 * RG, hipMemcpyDeviceToHost));
        }
        for (int64_t r = 0; r < R; ++r) {
          double v = finish_value(k, buf[live[r]], 1, t == PH_AGG_SUM);
          memcpy(dst + 8 * r, &v, 8);
        }
      }
    }
    res->key_types.resize(q->num_group_by);
    res->key_entry_size.resize(q->num_group_by);
    res->keys.resize(q->num_group_by);
    for (int g = 0; g < q->num_group_by; ++g) {
      const Dictionary& d = gdicts[g]->dict;
      const int32_t es = key_entry_size(d);
      res->key_types[g] = d.type;
      res->key_entry_size[g] = es;
      res->keys[g].assign((size_t)es * R, 0);
      for (int64_t r = 0; r < R; ++r) {
        const int64_t id = (key_of(r) / kp.group_stride[g]) % std::max<int64_t>(1, d.size);
        put_key_value(d, id, res->keys[g].data() + (size_t)es * r, es);
      }
    }
  }
  finish_fused();
  stats.num_entries_scanned_post_filter = stats.num_docs_scanned * ncols_proj;
  stamp("done");
  stats.host_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count() - dev_ms;
  return res.release();
}

}  // namespace ph
