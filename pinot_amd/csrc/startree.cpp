// startree.cpp -- star-tree (StarTreeV2) indexes: pinning a segment's star-tree beside it, choosing it for a query the
// way the reference's plan nodes do, the traversal on the host, and the query over the star-tree's records on the GPU.
//
//   load      StarTreeLoaderUtils / StarTreeIndexContainer (pinot-segment-local/.../startree/v2/store/): the STAR_TREE
//             buffer (OffHeapStarTree.java:45-83, OffHeapStarTreeNode.java:29-158) parsed on the host; the records'
//             dimension forward indexes (fixed-bit dictIds of the segment's dictionaries) and function-column pair
//             columns (raw LONG / DOUBLE) pinned as a segment of their own (the "view")
//   choose    GroupByPlanNode.java:77-99 / AggregationPlanNode.java:100-141 with StarTreeUtils.java:56-214: skipStarTree
//             unset; an aggregation-only query goes to FastFilteredCountOperator / NonScanBasedAggregationOperator
//             first; every aggregation a function-column pair of the tree; the filter an AND of per-column predicates
//             (an OR only over one column, no NOT); predicate and group-by columns all tree dimensions
//   traverse  StarTreeFilterOperator.traverseStarTree (:207-358): BFS, star nodes for dimensions without predicates
//             or group-by, aggregated documents once every predicate and group-by column is consumed, leaf ranges and
//             the remaining predicate columns otherwise
//   execute   the view with the query rewritten onto its pair columns (COUNT -> SUM(count__*), SUM / MIN / MAX(c)
//             -> SUM(sum__c) / MIN(min__c) / MAX(max__c)) and its filter = the traversal's documents AND the
//             remaining composites (StarTreeFilterOperator.getFilterOperator :157-199): the same kernels as any query;
//             the segments the star-tree does not serve run as usual and the two results merge by group value
#include <algorithm>
#include <cstring>
#include <functional>

#include "ph_internal.h"

ph_segment::~ph_segment() = default;

namespace ph {

ph_result* query_execute_impl(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg,
                              const DenseArgs* dn);

StarTree::~StarTree() {
  if (view) {
    star_tree_forget(*view->ctx, view);
    delete view;
  }
}

namespace {

constexpr uint64_t kStarMagic = 0xBADDA55B00DAD00Dull;
constexpr int32_t kAll = -1;  // StarTreeNode.ALL

inline int32_t le32(const uint8_t* p) {
  int32_t v;
  memcpy(&v, p, 4);
  return v;
}

// OffHeapStarTree(PinotDataBuffer): magic, version 1, root offset = header size, dimension (id, length, UTF-8 name)s,
// node count; the nodes fill the rest exactly
void parse_tree(const uint8_t* b, uint64_t size, std::vector<std::string>* dims, std::vector<int32_t>* nodes,
                int32_t* num_nodes) {
  if (!b || size < 24) fail(PH_ERR_INVALID_ARGUMENT, "star-tree buffer too small");
  uint64_t magic;
  memcpy(&magic, b, 8);
  if (magic != kStarMagic) fail(PH_ERR_INVALID_ARGUMENT, "invalid magic marker in star-tree data buffer");
  if (le32(b + 8) != 1) fail(PH_ERR_INVALID_ARGUMENT, "invalid version in star-tree data buffer");
  const int64_t root = le32(b + 12);
  const int32_t nd = le32(b + 16);
  if (nd <= 0 || nd > 64) fail(PH_ERR_INVALID_ARGUMENT, "star-tree dimension count");
  uint64_t off = 20;
  dims->assign((size_t)nd, std::string());
  for (int32_t i = 0; i < nd; ++i) {
    if (off + 8 > size) fail(PH_ERR_INVALID_ARGUMENT, "truncated star-tree header");
    const int32_t id = le32(b + off), len = le32(b + off + 4);
    off += 8;
    if (id < 0 || id >= nd || len < 0 || off + (uint64_t)len > size) fail(PH_ERR_INVALID_ARGUMENT, "star-tree dimension");
    (*dims)[id].assign(reinterpret_cast<const char*>(b + off), (size_t)len);
    off += (uint64_t)len;
  }
  if (off + 4 > size) fail(PH_ERR_INVALID_ARGUMENT, "truncated star-tree header");
  const int32_t n = le32(b + off);
  off += 4;
  if ((int64_t)off != root) fail(PH_ERR_INVALID_ARGUMENT, "error loading star-tree, header length mis-match");
  if (n <= 0 || off + (uint64_t)n * 28 != size) fail(PH_ERR_INVALID_ARGUMENT, "error loading star-tree, buffer size mis-match");
  nodes->resize((size_t)n * 7);
  for (int64_t i = 0; i < (int64_t)n * 7; ++i) (*nodes)[(size_t)i] = le32(b + off + 4 * i);
  *num_nodes = n;
  // the traversal's invariants: children are later nodes one dimension deeper, sorted by value
  for (int32_t i = 0; i < n; ++i) {
    const int32_t* x = nodes->data() + 7 * i;
    if (x[5] == -1) continue;
    if (x[5] <= i || x[6] < x[5] || x[6] >= n) fail(PH_ERR_INVALID_ARGUMENT, "star-tree child range");
    for (int32_t c = x[5]; c <= x[6]; ++c) {
      const int32_t* y = nodes->data() + 7 * c;
      if (y[0] != x[0] + 1 || y[0] >= nd) fail(PH_ERR_INVALID_ARGUMENT, "star-tree child dimension");
      if (c > x[5] && y[1] <= (nodes->data() + 7 * (c - 1))[1]) fail(PH_ERR_INVALID_ARGUMENT, "star-tree child order");
    }
  }
}

// AggregationFunctionColumnPair.toColumnName of a query aggregation (StarTreeUtils.extractAggregationFunctionPairs
// :56-71): "" when the aggregation is not a plain column (or *)
std::string pair_of(const ph_aggregation& a) {
  if (a.expr_op != PH_EXPR_NONE) return "";
  switch (a.type) {
    case PH_AGG_COUNT: return "count__*";
    case PH_AGG_SUM: return a.column ? std::string("sum__") + a.column : "";
    case PH_AGG_MIN: return a.column ? std::string("min__") + a.column : "";
    case PH_AGG_MAX: return a.column ? std::string("max__") + a.column : "";
    case PH_AGG_DISTINCTCOUNTHLL: return a.column ? std::string("distinctCountHLL__") + a.column : "";
  }
  return "";
}

// java.lang.String.hashCode over UTF-16 code units of a UTF-8 name
int32_t java_string_hash(const std::string& s) {
  uint32_t h = 0;
  for (size_t i = 0; i < s.size();) {
    const uint8_t c = (uint8_t)s[i];
    uint32_t cp = c, extra = 0;
    if (c >= 0xF0) { cp = c & 0x07; extra = 3; }
    else if (c >= 0xE0) { cp = c & 0x0F; extra = 2; }
    else if (c >= 0xC0) { cp = c & 0x1F; extra = 1; }
    ++i;
    for (uint32_t k = 0; k < extra && i < s.size(); ++k, ++i) cp = (cp << 6) | ((uint8_t)s[i] & 0x3F);
    if (cp >= 0x10000) {
      cp -= 0x10000;
      h = 31 * h + (0xD800 + (cp >> 10));
      h = 31 * h + (0xDC00 + (cp & 0x3FF));
    } else {
      h = 31 * h + cp;
    }
  }
  return (int32_t)h;
}

// java.util.HashSet<String> iteration order of names inserted in this order (no resize below 13 entries): by bucket
// (hash ^ hash >>> 16) & (capacity - 1), insertion order within a bucket
std::vector<std::string> hashset_order(const std::vector<std::string>& names) {
  int64_t cap = 16;
  while ((int64_t)names.size() > cap * 3 / 4) cap *= 2;
  std::vector<std::pair<uint32_t, size_t>> k;
  for (size_t i = 0; i < names.size(); ++i) {
    const uint32_t h = (uint32_t)java_string_hash(names[i]);
    k.push_back({(h ^ (h >> 16)) & (uint32_t)(cap - 1), i});
  }
  std::stable_sort(k.begin(), k.end(), [](auto& a, auto& b) { return a.first < b.first; });
  std::vector<std::string> out;
  for (auto& e : k) out.push_back(names[e.second]);
  return out;
}

// one predicate column of the star-tree filter: its composites (predicate indices ORed) and matching dictIds
struct ColPreds {
  std::string col;
  std::vector<std::vector<int32_t>> composites;
};

// StarTreeUtils.extractPredicateEvaluatorsMap (:85-134): false when the filter cannot be solved by a star-tree
bool extract_predicates(const ph_query* q, ph_segment* seg, std::vector<ColPreds>* out) {
  out->clear();
  if (q->filter_root < 0) return true;
  auto col_of = [&](const std::string& c) -> ColPreds& {
    for (auto& x : *out)
      if (x.col == c) return x;
    out->push_back(ColPreds{c, {}});
    return out->back();
  };
  auto evaluate = [&](int32_t pi, bool* at, bool* af) -> bool {
    if (pi < 0 || pi >= q->num_predicates) fail(PH_ERR_INVALID_ARGUMENT, "bad predicate index");
    const ph_predicate& p = q->predicates[pi];
    if (!p.column) fail(PH_ERR_BAD_QUERY, "predicate without column");
    auto it = seg->columns.find(p.column);
    if (it == seg->columns.end()) fail(PH_ERR_BAD_QUERY, std::string("Column not found: ") + p.column);
    if (it->second->is_raw) return false;  // "Star-tree does not support non-dictionary encoded dimension" (:260-263)
    predicate_dict_ids(p, *it->second, at, af);
    return true;
  };
  std::vector<int32_t> queue{q->filter_root};
  for (size_t h = 0; h < queue.size(); ++h) {
    const int32_t ni = queue[h];
    if (ni < 0 || ni >= q->num_filter_nodes) fail(PH_ERR_INVALID_ARGUMENT, "bad filter node index");
    const ph_filter_node& f = q->filter_nodes[ni];
    if (f.type == PH_FILTER_AND) {
      for (int i = 0; i < f.num_children; ++i) queue.push_back(f.children[i]);
    } else if (f.type == PH_FILTER_NOT) {
      return false;
    } else if (f.type == PH_FILTER_OR) {
      // isOrClauseValidForStarTree (:179-214): only predicates (nested ORs flattened) on one column
      std::vector<int32_t> preds;
      std::function<bool(int32_t)> flatten = [&](int32_t x) -> bool {
        const ph_filter_node& g = q->filter_nodes[x];
        for (int i = 0; i < g.num_children; ++i) {
          const int32_t c = g.children[i];
          if (c < 0 || c >= q->num_filter_nodes) fail(PH_ERR_INVALID_ARGUMENT, "bad filter node index");
          const ph_filter_node& k = q->filter_nodes[c];
          if (k.type == PH_FILTER_AND || k.type == PH_FILTER_NOT) return false;
          if (k.type == PH_FILTER_OR) {
            if (!flatten(c)) return false;
          } else {
            preds.push_back(k.predicate);
          }
        }
        return true;
      };
      if (!flatten(ni)) return false;
      std::string col;
      std::vector<int32_t> evs;
      bool always_true = false;
      for (int32_t pi : preds) {
        bool at = false, af = false;
        if (!evaluate(pi, &at, &af)) return false;
        if (at) {
          always_true = true;
          break;
        }
        if (af) continue;
        const std::string c = q->predicates[pi].column;
        if (col.empty()) col = c;
        else if (col != c) return false;
        evs.push_back(pi);
      }
      // an always-true OR, or one whose predicates are all always-false, adds nothing (NOTE at :107)
      if (!always_true && !evs.empty()) col_of(col).composites.push_back(evs);
    } else {
      bool at = false, af = false;
      if (!evaluate(f.predicate, &at, &af)) return false;
      if (!at) col_of(q->predicates[f.predicate].column).composites.push_back({f.predicate});
    }
  }
  return true;
}

// the first star-tree of the segment the query fits (isFitForStarTree, StarTreeUtils.java:144-169), or nullptr
StarTree* choose_tree(const ph_query* q, ph_segment* seg, std::vector<ColPreds>* preds) {
  if (seg->star_trees.empty() || q->skip_star_tree) return nullptr;
  std::vector<std::string> pairs;
  for (int k = 0; k < q->num_aggregations; ++k) {
    std::string p = pair_of(q->aggregations[k]);
    if (p.empty()) return nullptr;
    pairs.push_back(p);
  }
  if (pairs.empty()) return nullptr;
  // AggregationPlanNode: FastFilteredCountOperator and NonScanBasedAggregationOperator come first (:100-119)
  if (q->num_group_by == 0) {
    bool count_only = true, non_scan = q->filter_root < 0;
    for (int k = 0; k < q->num_aggregations; ++k) {
      count_only &= q->aggregations[k].type == PH_AGG_COUNT;
      non_scan &= q->aggregations[k].type != PH_AGG_SUM;
    }
    if (non_scan) return nullptr;
    if (count_only && q->filter_root >= 0 && filter_index_countable(q, seg)) return nullptr;
  }
  if (!extract_predicates(q, seg, preds)) return nullptr;
  for (auto& t : seg->star_trees) {
    bool fits = true;
    for (auto& p : pairs) fits = fits && std::find(t->pairs.begin(), t->pairs.end(), p) != t->pairs.end();
    auto is_dim = [&](const std::string& c) { return std::find(t->dims.begin(), t->dims.end(), c) != t->dims.end(); };
    for (int g = 0; g < q->num_group_by && fits; ++g) fits = q->group_by[g] && is_dim(q->group_by[g]);
    for (auto& c : *preds) fits = fits && is_dim(c.col);
    if (!fits) continue;
    for (auto& p : pairs)
      if (!t->served.count(p)) fail(PH_ERR_UNSUPPORTED, "star-tree pair " + p + " is not on the GPU path");
    return t.get();
  }
  return nullptr;
}

// StarTreeFilterOperator.traverseStarTree (:207-358) + getFilterOperator's AND (:157-199)
StarSegPlan traverse(const StarTree& t, ph_segment* seg, const ph_query* q, const std::vector<ColPreds>& preds) {
  StarSegPlan plan;
  const int32_t* N = t.nodes.data();
  auto node = [&](int32_t i) { return N + 7 * (size_t)i; };
  auto is_leaf = [&](int32_t i) { return node(i)[5] == -1; };
  std::vector<std::string> remaining;  // predicate columns (first-seen order)
  for (auto& c : preds) remaining.push_back(c.col);
  std::set<std::string> remaining_gb;
  for (int g = 0; g < q->num_group_by; ++g) remaining_gb.insert(q->group_by[g]);
  bool found_leaf = is_leaf(0);
  bool have_global = false;
  std::vector<std::string> global;
  if (found_leaf) {
    global = remaining;
    have_global = true;
  }
  auto in = [](const std::vector<std::string>& v, const std::string& s) {
    return std::find(v.begin(), v.end(), s) != v.end();
  };
  // getMatchingDictIds (:375-443): the AND of the column's composites, each the OR of its predicates' dictIds
  auto matching_ids = [&](const std::string& col) {
    const Column& c = *seg->columns.at(col);
    std::vector<char> ids;
    for (auto& pc : preds) {
      if (pc.col != col) continue;
      for (auto& comp : pc.composites) {
        std::vector<char> u((size_t)c.cardinality, 0);
        for (int32_t pi : comp) {
          bool at = false, af = false;
          std::vector<char> m = predicate_dict_ids(q->predicates[pi], c, &at, &af);
          for (size_t k = 0; k < u.size(); ++k) u[k] |= m[k];
        }
        if (ids.empty()) ids = u;
        else
          for (size_t k = 0; k < u.size(); ++k) ids[k] &= u[k];
      }
    }
    return ids;
  };
  std::vector<std::pair<int32_t, int32_t>> docs;  // [start, end)
  std::vector<int32_t> queue{0};
  int32_t cur_dim = -1;
  std::vector<char> matching;
  int64_t num_matching = -1;
  for (size_t h = 0; h < queue.size(); ++h) {
    const int32_t i = queue[h];
    const int32_t* x = node(i);
    const int32_t dim = x[0];
    if (dim > cur_dim) {
      const std::string& name = t.dims[(size_t)dim];
      remaining.erase(std::remove(remaining.begin(), remaining.end(), name), remaining.end());
      remaining_gb.erase(name);
      if (found_leaf && !have_global) {
        global = remaining;
        have_global = true;
      }
      num_matching = -1;
      cur_dim = dim;
    }
    if (remaining.empty() && remaining_gb.empty()) {
      docs.push_back({x[4], x[4] + 1});  // the aggregated document
      continue;
    }
    if (is_leaf(i)) {
      docs.push_back({x[2], x[3]});
      continue;
    }
    const std::string& child_dim = t.dims[(size_t)dim + 1];
    const int32_t first = x[5], last = x[6];
    int32_t star = -1;
    if ((!have_global || !in(global, child_dim)) && !remaining_gb.count(child_dim) && node(first)[1] == kAll) star = first;
    if (in(remaining, child_dim)) {
      if (num_matching < 0) {
        matching = matching_ids(child_dim);
        num_matching = 0;
        for (char m : matching) num_matching += m != 0;
        if (num_matching == 0) {
          plan.empty = true;
          return plan;
        }
      }
      auto match = [&](int32_t c) {
        const int32_t v = node(c)[1];
        return v >= 0 && v < (int32_t)matching.size() && matching[(size_t)v];
      };
      const int64_t nch = (int64_t)last - first + 1;
      if (num_matching * 10 > nch) {
        if (star >= 0 && num_matching >= nch - 1) {
          std::vector<int32_t> kids;
          bool kid_leaf = false;
          for (int32_t c = first; c <= last; ++c)
            if (match(c)) {
              kids.push_back(c);
              kid_leaf |= is_leaf(c);
            }
          if ((int64_t)kids.size() == nch - 1) {  // every non-star child matches: the star node
            queue.push_back(star);
            found_leaf |= is_leaf(star);
          } else {
            queue.insert(queue.end(), kids.begin(), kids.end());
            found_leaf |= kid_leaf;
          }
        } else {
          for (int32_t c = first; c <= last; ++c)
            if (match(c)) {
              queue.push_back(c);
              found_leaf |= is_leaf(c);
            }
        }
      } else {  // binary search per matching dictId (getChildForDimensionValue)
        for (int32_t v = 0; v < (int32_t)matching.size(); ++v) {
          if (!matching[(size_t)v]) continue;
          int32_t lo = first, hi = last;
          while (lo <= hi) {
            const int32_t mid = (lo + hi) / 2, mv = node(mid)[1];
            if (mv == v) {
              queue.push_back(mid);
              found_leaf |= is_leaf(mid);
              break;
            }
            if (mv < v) lo = mid + 1;
            else hi = mid - 1;
          }
        }
      }
    } else if (star >= 0) {
      queue.push_back(star);
      found_leaf |= is_leaf(star);
    } else {
      for (int32_t c = first; c <= last; ++c)
        if (node(c)[1] != kAll) {
          queue.push_back(c);
          found_leaf |= is_leaf(c);
        }
    }
  }
  // the matched documents as a MutableRoaringBitmap holds them: sorted, merged
  std::sort(docs.begin(), docs.end());
  for (auto& d : docs) {
    if (d.second <= d.first) continue;
    if (!plan.ranges.empty() && plan.ranges.back() + 1 >= d.first) {
      plan.ranges.back() = std::max(plan.ranges.back(), d.second - 1);
    } else {
      plan.ranges.push_back(d.first);
      plan.ranges.push_back(d.second - 1);
    }
  }
  if (plan.ranges.empty()) plan.empty = true;
  // the remaining predicate columns (globalRemainingPredicateColumns, a HashSet<String>), their composites in the
  // predicate map's order
  std::vector<std::string> rem;
  for (auto& c : preds)
    if (have_global && in(global, c.col)) rem.push_back(c.col);
  for (auto& col : hashset_order(rem))
    for (auto& c : preds)
      if (c.col == col)
        for (auto& comp : c.composites) plan.composites.push_back(comp);
  return plan;
}

}  // namespace

bool star_tree_serves_any(const ph_query* q, ph_segment* const* segs, int32_t nseg) {
  if (!q || q->skip_star_tree) return false;
  std::vector<ColPreds> preds;
  for (int32_t i = 0; i < nseg; ++i)
    if (segs[i] && !segs[i]->star_trees.empty() && choose_tree(q, segs[i], &preds)) return true;
  return false;
}

ph_result* star_tree_execute(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg, int dense_op) {
  if (!q || q->skip_star_tree || nseg <= 0 || q->num_aggregations <= 0) return nullptr;
  std::vector<ph_segment*> plain, views;
  std::map<const ph_segment*, StarSegPlan> plans;
  std::vector<ColPreds> preds;
  int64_t star_total_docs = 0;
  for (int32_t i = 0; i < nseg; ++i) {
    ph_segment* s = segs[i];
    StarTree* t = (s && !s->star_trees.empty()) ? choose_tree(q, s, &preds) : nullptr;
    if (!t) {
      plain.push_back(s);
      continue;
    }
    if (dense_op) fail(PH_ERR_UNSUPPORTED, "star-tree segments on dense partials");
    plans[t->view] = traverse(*t, s, q, preds);
    views.push_back(t->view);
    star_total_docs += s->num_docs;
  }
  if (views.empty()) return nullptr;
  // the query over the views: the aggregations on their pair columns (a COUNT reads back as a SUM of counts)
  ph_query q2 = *q;
  q2.skip_star_tree = 1;
  std::vector<ph_aggregation> aggs((size_t)q->num_aggregations);
  std::vector<std::string> cols((size_t)q->num_aggregations);
  for (int k = 0; k < q->num_aggregations; ++k) {
    aggs[k] = q->aggregations[k];
    cols[k] = pair_of(q->aggregations[k]);
    aggs[k].column = cols[k].c_str();
    if (aggs[k].type == PH_AGG_COUNT) aggs[k].type = PH_AGG_SUM;
  }
  q2.aggregations = aggs.data();
  q2.min_segment_group_trim_size = 0;  // (a trimmed query runs one segment per call: segment_trim_execute)
  DenseArgs da{0, nullptr, 0, 0, nullptr};
  da.star = &plans;
  std::unique_ptr<ph_result> rs(query_execute_impl(ctx, &q2, views.data(), (int32_t)views.size(), &da));
  // COUNT intermediate results are longs: the SUM of the count__* column read back (exact: an integer SUM)
  for (int k = 0; k < q->num_aggregations; ++k) {
    rs->agg_types[(size_t)k] = q->aggregations[k].type;
    if (q->aggregations[k].type != PH_AGG_COUNT) continue;
    uint8_t* p = rs->aggs[(size_t)k].data();
    for (int64_t g = 0; g < rs->num_groups; ++g) {
      double d;
      memcpy(&d, p + 8 * g, 8);
      const int64_t v = (int64_t)d;
      memcpy(p + 8 * g, &v, 8);
    }
  }
  rs->stats.num_total_docs = star_total_docs;
  rs->stats.num_segments_star_tree = (int64_t)views.size();
  if (plain.empty()) return rs.release();
  ph_query q1 = *q;
  q1.skip_star_tree = 1;
  std::unique_ptr<ph_result> rp(query_execute_impl(ctx, &q1, plain.data(), (int32_t)plain.size(), nullptr));
  std::vector<std::unique_ptr<ph_result>> parts;
  const double ms = rp->stats.device_ms + rs->stats.device_ms;  // (the two calls ran one after the other)
  parts.push_back(std::move(rp));
  parts.push_back(std::move(rs));
  ph_result* r = merge_results_by_value(q, parts);  // statistics summed by the merge
  r->stats.device_ms = ms;
  return r;
}

// ph_segment_add_star_tree: the view holds the dimensions (the segment's dictionaries re-serialised for the pin) and
// the count / sum / min / max pair columns (raw: dictionary-encoded at pin like any raw column)
void star_tree_add_impl(ph_segment* seg, const ph_star_tree_desc* d) {
  if (!seg || !d) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
  if (seg->parent_docs >= 0) fail(PH_ERR_INVALID_ARGUMENT, "a star-tree view has no star-trees");
  auto t = std::make_unique<StarTree>();
  parse_tree(static_cast<const uint8_t*>(d->tree), d->tree_size, &t->dims, &t->nodes, &t->num_nodes);
  if (d->num_docs < 0) fail(PH_ERR_INVALID_ARGUMENT, "star-tree num_docs");
  if (d->num_dimensions != (int32_t)t->dims.size() || !d->dimensions || !d->dimension_forward_index ||
      !d->dimension_forward_index_size)
    fail(PH_ERR_INVALID_ARGUMENT, "star-tree dimensions do not match the tree");
  for (int32_t i = 0; i < d->num_dimensions; ++i)
    if (!d->dimensions[i] || t->dims[(size_t)i] != d->dimensions[i])
      fail(PH_ERR_INVALID_ARGUMENT, "star-tree dimension order differs from the tree's split order");
  // the documents a node names must be records of the tree
  for (int32_t i = 0; i < t->num_nodes; ++i) {
    const int32_t* x = t->nodes.data() + 7 * i;
    if (x[4] < 0 || x[4] >= d->num_docs) fail(PH_ERR_INVALID_ARGUMENT, "star-tree aggregated document out of range");
    if (x[5] == -1 && (x[2] < 0 || x[3] < x[2] || x[3] > d->num_docs))
      fail(PH_ERR_INVALID_ARGUMENT, "star-tree leaf documents out of range");
  }
  std::vector<ph_column_desc> cols;
  std::vector<std::vector<uint8_t>> dict_bytes;
  dict_bytes.reserve((size_t)d->num_dimensions);
  for (int32_t i = 0; i < d->num_dimensions; ++i) {
    auto it = seg->columns.find(d->dimensions[i]);
    if (it == seg->columns.end()) fail(PH_ERR_INVALID_ARGUMENT, std::string("star-tree dimension not pinned: ") + d->dimensions[i]);
    const Column& c = *it->second;
    if (c.is_raw) fail(PH_ERR_INVALID_ARGUMENT, "star-tree dimension " + c.name + " has no dictionary");
    // the dictionary as SegmentDictionaryCreator wrote it (big-endian fixed width; STRING zero-padded)
    const Dictionary& dict = c.dict;
    int w = dict.type == PH_INT || dict.type == PH_FLOAT ? 4 : 8;
    if (dict.type == PH_STRING) w = std::max(1, dict.max_string_len);
    std::vector<uint8_t> b((size_t)w * (size_t)std::max<int64_t>(1, dict.size), 0);
    for (int64_t k = 0; k < dict.size; ++k) {
      uint8_t* o = b.data() + (size_t)w * k;
      uint64_t u = 0;
      switch (dict.type) {
        case PH_INT: u = (uint32_t)(int32_t)dict.ints[k]; break;
        case PH_LONG: u = (uint64_t)dict.ints[k]; break;
        case PH_FLOAT: { float f = (float)dict.reals[k]; uint32_t v; memcpy(&v, &f, 4); u = v; break; }
        case PH_DOUBLE: memcpy(&u, &dict.reals[k], 8); break;
        default: memcpy(o, dict.strings[k].data(), dict.strings[k].size()); continue;
      }
      for (int j = 0; j < w; ++j) o[j] = (uint8_t)(u >> (8 * (w - 1 - j)));
    }
    dict_bytes.push_back(std::move(b));
    ph_column_desc cd{};
    cd.name = d->dimensions[i];
    cd.data_type = c.data_type;
    cd.cardinality = c.cardinality;
    cd.bits_per_element = c.bits;
    cd.forward_index = d->dimension_forward_index[i];
    cd.forward_index_size = d->dimension_forward_index_size[i];
    cd.dictionary = dict_bytes.back().data();
    cd.dictionary_size = dict_bytes.back().size();
    cd.dictionary_entry_size = w;
    cols.push_back(cd);
  }
  for (int32_t i = 0; i < d->num_metrics; ++i) {
    if (!d->metrics || !d->metrics[i]) fail(PH_ERR_INVALID_ARGUMENT, "star-tree metric without a name");
    const std::string name = d->metrics[i];
    t->pairs.push_back(name);
    const size_t sep = name.find("__");
    const std::string fn = sep == std::string::npos ? name : name.substr(0, sep);
    const bool ours = fn == "count" || fn == "sum" || fn == "min" || fn == "max";
    if (!ours || !d->metric_forward_index || !d->metric_forward_index[i]) continue;
    ph_column_desc cd{};
    cd.name = d->metrics[i];
    cd.data_type = fn == "count" ? PH_LONG : PH_DOUBLE;  // ValueAggregator.getAggregatedValueType
    cd.forward_index = d->metric_forward_index[i];
    cd.forward_index_size = d->metric_forward_index_size ? d->metric_forward_index_size[i] : 0;
    cd.raw_forward_index = 1;
    cols.push_back(cd);
    t->served.insert(name);
  }
  ph_segment_desc vd{};
  const std::string vname = seg->name + "#startree" + std::to_string(seg->star_trees.size());
  vd.name = vname.c_str();
  vd.num_docs = d->num_docs;
  vd.num_columns = (int32_t)cols.size();
  vd.columns = cols.data();
  ph_segment* v = segment_pin_impl(seg->ctx, &vd);
  v->parent_docs = seg->num_docs;
  t->view = v;
  seg->device_bytes += v->device_bytes;
  seg->star_trees.push_back(std::move(t));
}

void star_tree_check_impl(const void* tree, uint64_t size, int32_t* num_nodes, int32_t* num_dimensions) {
  std::vector<std::string> dims;
  std::vector<int32_t> nodes;
  int32_t n = 0;
  parse_tree(static_cast<const uint8_t*>(tree), size, &dims, &nodes, &n);
  if (num_nodes) *num_nodes = n;
  if (num_dimensions) *num_dimensions = (int32_t)dims.size();
}

}  // namespace ph
