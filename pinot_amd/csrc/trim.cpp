// trim.cpp -- segment group trim (GroupByOperator.java:114-130) for ph_query_execute.
//
// With a group-by, ORDER BY and minSegmentGroupTrimSize > 0, the reference trims every segment's groups to
// GroupByUtils.getTableCapacity(limit, minSegmentGroupTrimSize) = max(5 * limit, min) (GroupByUtils.java:40-42)
// before the combine: TableResizer.trimInSegmentResults (TableResizer.java:321-343) fills a heap with the first
// `size` groups of the segment's group-key iterator, orders it with the reversed ORDER BY comparator (makeHeap /
// downHeap, :233-262) and replaces the heap top with every later group that compares greater; the kept groups' partial
// aggregates are what GroupByCombineOperator merges (IndexedTable upsert -> AggregationFunction.merge).
//
// Here each segment runs as its own query on the GPU (the one-launch combine over all segments cannot drop a
// segment's groups), its rows are put in the iterator order of the reference's ArrayBasedHolder -- ascending raw key
// over the segment's dictIds, column 0 least significant (DictionaryBasedGroupKeyGenerator.java:254-377) -- and
// trimmed by the same heap; the kept rows of all segments are merged on the host.  When the segment's cardinality
// product exceeds the ArrayBased threshold the reference iterates a hash map instead (IntGroupIdMap slot order /
// fastutil order); the kept set is the same unless ORDER BY values tie at the trim boundary.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "ph_internal.h"

namespace ph {

ph_result* query_execute_impl(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg,
                              const DenseArgs* dn);

namespace {

// clearspring HyperLogLog.cardinality() (stream 2.7.0; DistinctCountHLLAggregationFunction.extractFinalResult
// :362-364) over 1-byte registers: alpha_m m^2 / sum 2^-r, linear counting m ln(m / zeros) at or below 5m/2, Java
// Math.round (an empty register set's ln(inf) rounds to Long.MAX_VALUE)
int64_t hll_cardinality(const uint8_t* reg, int log2m) {
  const int64_t m = (int64_t)1 << log2m;
  double sum = 0, zeros = 0;
  for (int64_t j = 0; j < m; ++j) {
    sum += 1.0 / (double)(1LL << reg[j]);
    if (reg[j] == 0) zeros += 1;
  }
  const double mm = (double)m * (double)m;
  const double alpha_mm = log2m == 4 ? 0.673 * mm : log2m == 5 ? 0.697 * mm : log2m == 6 ? 0.709 * mm
                                                                                 : (0.7213 / (1 + 1.079 / m)) * mm;
  const double est = alpha_mm * (1 / sum);
  const double x = est <= 2.5 * (double)m ? (double)m * std::log((double)m / zeros) : est;
  if (std::isnan(x)) return 0;
  if (x >= 9.2233720368547758e18) return INT64_MAX;
  return (int64_t)std::floor(x + 0.5);
}

// Java's Double.compare / Float.compare order (NaN largest, -0.0 < 0.0): the natural order of the boxed values
int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x, y;
  memcpy(&x, &a, 8);
  memcpy(&y, &b, 8);
  if (std::isnan(a)) x = 0x7ff8000000000000LL;
  if (std::isnan(b)) y = 0x7ff8000000000000LL;
  return x == y ? 0 : (x < y ? -1 : 1);
}

// Java String.compareTo: UTF-16 code-unit order (UTF-8 byte order differs for supplementary-plane characters
// against U+E000..U+FFFF)
std::u16string utf16_of(const std::string& s) {
  std::u16string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    const uint8_t c = (uint8_t)s[i];
    uint32_t cp = c, n = 0;
    if (c >= 0xf0) { cp = c & 0x07; n = 3; }
    else if (c >= 0xe0) { cp = c & 0x0f; n = 2; }
    else if (c >= 0xc0) { cp = c & 0x1f; n = 1; }
    ++i;
    for (uint32_t k = 0; k < n && i < s.size(); ++k, ++i) cp = (cp << 6) | ((uint8_t)s[i] & 0x3f);
    if (cp >= 0x10000) {
      cp -= 0x10000;
      out.push_back((char16_t)(0xd800 + (cp >> 10)));
      out.push_back((char16_t)(0xdc00 + (cp & 0x3ff)));
    } else {
      out.push_back((char16_t)cp);
    }
  }
  return out;
}

int java_string_compare(const std::string& a, const std::string& b) {
  const std::u16string x = utf16_of(a), y = utf16_of(b);
  return x < y ? -1 : (x > y ? 1 : 0);
}

struct Row {
  // per group-by column the value's bytes: numeric types at their fixed width, STRING without its zero padding (a
  // segment-local query pads to its own max_string_len, so widths differ between segments)
  std::vector<std::string> kv;
  std::string key;          // merge key: the values, each length-prefixed
  std::vector<double> d;    // per aggregation: SUM/MIN/MAX value (COUNT in c)
  std::vector<int64_t> c;   // per aggregation: COUNT
  std::vector<std::vector<uint8_t>> hll;
  std::vector<int64_t> hc;  // per aggregation: a DISTINCTCOUNTHLL order-by value (its cardinality), set for the trim
  uint64_t raw = 0;         // ArrayBasedHolder raw key over the segment's dictIds
};

// Results of one query merged keyed by group VALUES -- GroupByCombineOperator / IndexedTable upsert with
// AggregationFunction.merge (GroupByCombineOperator.java:169-181, AggregationResultsBlockMerger.java:33-45): the
// segment-trim combine below and the multi-device combine's host path (multi.cpp)
class ValueMerge {
 public:
  explicit ValueMerge(const ph_query* q) : q_(q), ng_(q->num_group_by), na_(q->num_aggregations), key_size_(ng_, 0) {}

  // the shape (types, widths) and the statistics of one more result
  void note(const ph_result& r, bool add_device_ms = true) {
    ph_exec_stats& st = out_->stats;
    const ph_exec_stats& rs = r.stats;
    st.num_docs_scanned += rs.num_docs_scanned;
    st.num_entries_scanned_in_filter += rs.num_entries_scanned_in_filter;
    st.num_entries_scanned_post_filter += rs.num_entries_scanned_post_filter;
    st.num_total_docs += rs.num_total_docs;
    st.num_segments_processed += rs.num_segments_processed;
    st.num_segments_matched += rs.num_segments_matched;
    st.num_segments_star_tree += rs.num_segments_star_tree;
    st.num_groups_limit_reached |= rs.num_groups_limit_reached;
    st.sum_precision_flag |= rs.sum_precision_flag;
    st.device_ms = add_device_ms ? st.device_ms + rs.device_ms : std::max(st.device_ms, rs.device_ms);
    st.host_ms += rs.host_ms;
    st.plan_mode = rs.plan_mode;
    st.scan_kernel = rs.scan_kernel;
    st.limit_pass = std::max(st.limit_pass, rs.limit_pass);
    if (!typed_) {
      out_->key_types = r.key_types;
      out_->agg_types = r.agg_types;
      out_->agg_log2m = r.agg_log2m;
      out_->mode = r.mode;
      typed_ = true;
    }
    for (int c = 0; c < ng_ && c < (int)r.key_entry_size.size(); ++c) key_size_[c] = std::max(key_size_[c], r.key_entry_size[c]);
  }

  // r's groups as rows; with `seg`, each row also gets its ArrayBasedHolder raw key over seg's dictIds
  std::vector<Row> rows(const ph_result& r, const ph_segment* seg) const {
    const int64_t n = r.num_groups;
    std::vector<Row> out((size_t)n);
    for (int64_t g = 0; g < n; ++g) {
      Row& row = out[(size_t)g];
      uint64_t mult = 1;
      for (int c = 0; c < ng_; ++c) {
        const int w = r.key_entry_size[c];
        const uint8_t* kp = r.keys[c].data() + (size_t)g * w;
        const size_t len = r.key_types[c] == PH_STRING ? strnlen(reinterpret_cast<const char*>(kp), (size_t)w) : (size_t)w;
        row.kv.emplace_back(reinterpret_cast<const char*>(kp), len);
        const uint32_t l32 = (uint32_t)len;
        row.key.append(reinterpret_cast<const char*>(&l32), 4);
        row.key.append(row.kv.back());
        if (!seg) continue;
        // the key's dictId in this segment's dictionary (ArrayBasedHolder raw key)
        const Dictionary& d = seg->columns.at(q_->group_by[c])->dict;
        int64_t id = 0;
        switch (r.key_types[c]) {
          case PH_INT: { int32_t v; memcpy(&v, kp, 4); id = std::lower_bound(d.ints.begin(), d.ints.end(), (int64_t)v) - d.ints.begin(); break; }
          case PH_LONG: { int64_t v; memcpy(&v, kp, 8); id = std::lower_bound(d.ints.begin(), d.ints.end(), v) - d.ints.begin(); break; }
          case PH_FLOAT: {
            float v; memcpy(&v, kp, 4);
            id = std::lower_bound(d.reals.begin(), d.reals.end(), (double)v, [](double a, double b) { return java_double_compare(a, b) < 0; }) - d.reals.begin();
            break;
          }
          case PH_DOUBLE: {
            double v; memcpy(&v, kp, 8);
            id = std::lower_bound(d.reals.begin(), d.reals.end(), v, [](double a, double b) { return java_double_compare(a, b) < 0; }) - d.reals.begin();
            break;
          }
          default: id = std::lower_bound(d.strings.begin(), d.strings.end(), row.kv.back()) - d.strings.begin();
        }
        row.raw += (uint64_t)id * mult;
        mult *= (uint64_t)std::max<int64_t>(1, d.size);
      }
      row.d.assign((size_t)na_, 0.0);
      row.c.assign((size_t)na_, 0);
      row.hll.resize((size_t)na_);
      for (int k = 0; k < na_; ++k) {
        const int t = r.agg_types[k];
        const uint8_t* ap = r.aggs[k].data();
        if (t == PH_AGG_COUNT) {
          memcpy(&row.c[k], ap + 8 * g, 8);
        } else if (t == PH_AGG_DISTINCTCOUNTHLL) {
          const size_t m = (size_t)1 << r.agg_log2m[k];
          row.hll[k].assign(ap + m * g, ap + m * (g + 1));
        } else {
          memcpy(&row.d[k], ap + 8 * g, 8);
        }
      }
    }
    return out;
  }

  // GroupByCombineOperator: merge into the server table (AggregationFunction.merge)
  void add(std::vector<Row>& rows) {
    for (auto& row : rows) {
      auto it = index_.find(row.key);
      if (it == index_.end()) {
        index_.emplace(row.key, merged_.size());
        merged_.push_back(std::move(row));
        continue;
      }
      Row& dst = merged_[it->second];
      for (int k = 0; k < na_; ++k) {
        const int t = out_->agg_types[k];
        if (t == PH_AGG_COUNT) dst.c[k] += row.c[k];
        else if (t == PH_AGG_SUM) dst.d[k] += row.d[k];
        else if (t == PH_AGG_MIN) dst.d[k] = std::min(dst.d[k], row.d[k]);
        else if (t == PH_AGG_MAX) dst.d[k] = std::max(dst.d[k], row.d[k]);
        else
          for (size_t i = 0; i < dst.hll[k].size(); ++i) dst.hll[k][i] = std::max(dst.hll[k][i], row.hll[k][i]);
      }
    }
  }

  bool typed() const { return typed_; }
  ph_exec_stats& stats() { return out_->stats; }

  // the combined rows as a result (host vectors)
  ph_result* finish() {
    const int64_t R = (int64_t)merged_.size();
    out_->num_groups = R;
    out_->keys.resize((size_t)ng_);
    out_->aggs.resize((size_t)na_);
    out_->key_entry_size = key_size_;
    for (int c = 0; c < ng_; ++c) {
      const size_t w = (size_t)key_size_[c];
      out_->keys[c].assign(w * R, 0);
      for (int64_t g = 0; g < R; ++g) {
        const std::string& v = merged_[(size_t)g].kv[c];
        memcpy(out_->keys[c].data() + w * g, v.data(), std::min(w, v.size()));
      }
    }
    for (int k = 0; k < na_; ++k) {
      const int t = out_->agg_types[k];
      if (t == PH_AGG_DISTINCTCOUNTHLL) {
        const size_t m = (size_t)1 << out_->agg_log2m[k];
        out_->aggs[k].assign(m * R, 0);
        for (int64_t g = 0; g < R; ++g) memcpy(out_->aggs[k].data() + m * g, merged_[(size_t)g].hll[k].data(), m);
      } else {
        out_->aggs[k].assign(8 * (size_t)R, 0);
        for (int64_t g = 0; g < R; ++g) {
          if (t == PH_AGG_COUNT) memcpy(out_->aggs[k].data() + 8 * g, &merged_[(size_t)g].c[k], 8);
          else memcpy(out_->aggs[k].data() + 8 * g, &merged_[(size_t)g].d[k], 8);
        }
      }
    }
    return out_.release();
  }

 private:
  const ph_query* q_;
  int ng_, na_;
  std::vector<int32_t> key_size_;
  bool typed_ = false;
  std::unordered_map<std::string, size_t> index_;
  std::vector<Row> merged_;
  std::unique_ptr<ph_result> out_ = std::make_unique<ph_result>();
};

}  // namespace

ph_result* segment_trim_execute(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg) {
  const int ng = q->num_group_by, na = q->num_aggregations;
  for (int k = 0; k < q->num_order_by; ++k) {
    const ph_order_by& o = q->order_by[k];
    if (o.kind == PH_ORDER_AGGREGATION) {
      if (o.index < 0 || o.index >= na) fail(PH_ERR_BAD_QUERY, "ORDER BY aggregation index");
    } else if (o.index < 0 || o.index >= ng) {
      fail(PH_ERR_BAD_QUERY, "ORDER BY group-by index");
    }
  }
  const int64_t trim = std::max<int64_t>((int64_t)q->limit * 5, q->min_segment_group_trim_size);
  ph_query one = *q;
  one.min_segment_group_trim_size = 0;
  ValueMerge vm(q);
  for (int32_t s = 0; s < nseg; ++s) {
    // each segment on its own device's context (a multi-device ph_ctx pins segments on different GPUs)
    std::unique_ptr<ph_result> r(query_execute_impl(segs[s]->ctx, &one, segs + s, 1, nullptr));
    vm.note(*r);
    std::vector<Row> rows = vm.rows(*r, segs[s]);
    if ((int64_t)rows.size() > trim) {
      // an aggregation orders by its extractFinalResult (TableResizer.AggregationFunctionExtractor :425-447): a
      // DISTINCTCOUNTHLL by HyperLogLog.cardinality(), a long -- computed once per row
      for (int k = 0; k < q->num_order_by; ++k) {
        const ph_order_by& o = q->order_by[k];
        if (o.kind != PH_ORDER_AGGREGATION || r->agg_types[o.index] != PH_AGG_DISTINCTCOUNTHLL) continue;
        const int log2m = q->aggregations[o.index].log2m > 0 ? q->aggregations[o.index].log2m : 8;
        for (auto& row : rows) {
          row.hc.resize((size_t)na, 0);
          row.hc[o.index] = hll_cardinality(row.hll[o.index].data(), log2m);
        }
      }
      // TableResizer: the intermediate-record comparator over the ORDER BY values, reversed for the heap
      auto cmp_inter = [&](const Row& a, const Row& b) -> int {
        for (int k = 0; k < q->num_order_by; ++k) {
          const ph_order_by& o = q->order_by[k];
          int c = 0;
          if (o.kind == PH_ORDER_AGGREGATION) {
            const int j = o.index;
            if (r->agg_types[j] == PH_AGG_COUNT) c = a.c[j] < b.c[j] ? -1 : (a.c[j] > b.c[j] ? 1 : 0);
            else if (r->agg_types[j] == PH_AGG_DISTINCTCOUNTHLL) c = a.hc[j] < b.hc[j] ? -1 : (a.hc[j] > b.hc[j] ? 1 : 0);
            else c = java_double_compare(a.d[j], b.d[j]);
          } else {
            const uint8_t* pa = reinterpret_cast<const uint8_t*>(a.kv[o.index].data());
            const uint8_t* pb = reinterpret_cast<const uint8_t*>(b.kv[o.index].data());
            switch (r->key_types[o.index]) {
              case PH_INT: { int32_t x, y; memcpy(&x, pa, 4); memcpy(&y, pb, 4); c = x < y ? -1 : (x > y ? 1 : 0); break; }
              case PH_LONG: { int64_t x, y; memcpy(&x, pa, 8); memcpy(&y, pb, 8); c = x < y ? -1 : (x > y ? 1 : 0); break; }
              case PH_FLOAT: { float x, y; memcpy(&x, pa, 4); memcpy(&y, pb, 4); c = java_double_compare(x, y); break; }
              case PH_DOUBLE: { double x, y; memcpy(&x, pa, 8); memcpy(&y, pb, 8); c = java_double_compare(x, y); break; }
              default: c = java_string_compare(a.kv[o.index], b.kv[o.index]);
            }
          }
          if (!o.asc) c = -c;
          if (c) return c;
        }
        return 0;
      };
      auto cmp = [&](const Row* a, const Row* b) { return cmp_inter(*b, *a); };  // reversed
      std::vector<const Row*> order;
      order.reserve(rows.size());
      for (auto& row : rows) order.push_back(&row);
      std::stable_sort(order.begin(), order.end(), [](const Row* a, const Row* b) { return a->raw < b->raw; });
      const int64_t size = trim;
      std::vector<const Row*> heap(order.begin(), order.begin() + size);
      auto down_heap = [&](int64_t i) {  // TableResizer.downHeap (fastutil ObjectHeaps)
        const Row* e = heap[(size_t)i];
        int64_t child;
        while ((child = (i << 1) + 1) < size) {
          const Row* t = heap[(size_t)child];
          const int64_t right = child + 1;
          if (right < size && cmp(heap[(size_t)right], t) < 0) {
            child = right;
            t = heap[(size_t)child];
          }
          if (cmp(e, t) <= 0) break;
          heap[(size_t)i] = t;
          i = child;
        }
        heap[(size_t)i] = e;
      };
      for (int64_t i = size >> 1; i-- != 0;) down_heap(i);  // makeHeap
      for (size_t x = (size_t)size; x < order.size(); ++x) {
        if (cmp(order[x], heap[0]) > 0) {
          heap[0] = order[x];
          down_heap(0);
        }
      }
      std::vector<Row> kept;
      kept.reserve((size_t)size);
      for (const Row* h : heap) kept.push_back(*h);
      rows.swap(kept);
    }
    vm.add(rows);
  }
  if (!vm.typed()) {  // no segment: an empty result with the query's shape
    std::unique_ptr<ph_result> r(query_execute_impl(ctx, &one, segs, 0, nullptr));
    return r.release();
  }
  return vm.finish();
}

// the multi-device combine's host path: per-device results of one query merged by group values (device_ms: the
// slowest device's)
ph_result* merge_results_by_value(const ph_query* q, const std::vector<std::unique_ptr<ph_result>>& parts) {
  ValueMerge vm(q);
  for (auto& r : parts) {
    vm.note(*r, false);
    std::vector<Row> rows = vm.rows(*r, nullptr);
    vm.add(rows);
  }
  return vm.finish();
}

}  // namespace ph
