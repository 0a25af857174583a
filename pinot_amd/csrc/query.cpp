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
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <set>
#include <unordered_map>

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
  std::vector<PNode> kids;
};

struct BitmapLeaf {
  ph_segment* seg;
  Column* col;
  std::vector<int32_t> dict_ids;
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

DictIdSet evaluate_predicate(const ph_predicate& p, const Column& c) {
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
      std::set<int32_t> ids;
      for (int i = 0; i < p.num_values; ++i) {
        int64_t id = d.index_of(lit(p.values[i]));
        if (id >= 0) ids.insert((int32_t)id);
      }
      if (p.type == PH_PRED_IN) {
        if (ids.empty()) { r.always_false = true; return r; }
        if ((int64_t)ids.size() == card) { r.always_true = true; return r; }
        r.ids.assign(ids.begin(), ids.end());
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
      r.ids.assign(ids.begin(), ids.end());
      return r;
    }
    case PH_PRED_RANGE: {
      const std::string lo = lit(p.lower), hi = lit(p.upper);
      int64_t start, end;
      if (lo == "*" || lo.empty()) {
        start = 0;
      } else {
        int64_t ii = d.insertion_index_of(lo);
        start = ii < 0 ? -(ii + 1) : (p.lower_inclusive ? ii : ii + 1);
      }
      if (hi == "*" || hi.empty()) {
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
        inv.kids.push_back(std::move(n));
        return inv;
      }
      return n;
    }
    n.scan = true;
    n.col = sl;
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

int count_scan_leaves(const PNode& n) {
  if (n.kind != L_NODE) return 0;
  int s = n.scan ? 1 : 0;
  for (auto& k : n.kids) s += count_scan_leaves(k);
  return s;
}

// host-side storage of a segment's program before device upload
struct SegProgram {
  std::vector<FilterInsn> insns;
  std::vector<std::pair<size_t, std::vector<uint32_t>>> payloads;  // insn index -> words (set / ranges)
  std::vector<std::pair<size_t, int>> bitmap_refs;                 // insn index -> bitmap leaf
  int depth = 0, max_depth = 0;
};

void emit(const PNode& n, SegProgram& p) {
  FilterInsn in{};
  if (n.op == OP_AND || n.op == OP_OR || n.op == OP_NOT) {
    for (auto& k : n.kids) emit(k, p);
    in.op = n.op;
    in.col = (int32_t)n.kids.size();
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

// ------------------------------------------------------------------ roaring container directory
struct RoaringView {
  std::vector<RoaringContainer> containers;
};

uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t be32u(const uint8_t* p) { return ((uint32_t)p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3]; }

// Parse one portable-format RoaringBitmap (RoaringFormatSpec; RoaringBitmap 0.9.38 serialize()).
void parse_roaring(const uint8_t* blob, uint64_t len, uint64_t blob_offset, std::vector<RoaringContainer>& out) {
  if (len < 4) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated bitmap");
  const uint32_t cookie = le32(blob);
  uint64_t pos = 4;
  uint32_t size;
  const uint8_t* run_flags = nullptr;
  bool has_offsets;
  if ((cookie & 0xFFFF) == 12347) {  // SERIAL_COOKIE: run containers present
    size = (cookie >> 16) + 1;
    run_flags = blob + pos;
    pos += (size + 7) / 8;
    has_offsets = size >= 4;  // NO_OFFSET_THRESHOLD
  } else if (cookie == 12346) {  // SERIAL_COOKIE_NO_RUNCONTAINER
    size = le32(blob + pos);
    pos += 4;
    has_offsets = true;
  } else {
    fail(PH_ERR_INVALID_ARGUMENT, "inverted index: bad roaring cookie");
  }
  const uint8_t* desc = blob + pos;
  pos += 4ull * size;
  const uint8_t* offs = nullptr;
  if (has_offsets) {
    offs = blob + pos;
    pos += 4ull * size;
  }
  if (pos > len) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated roaring header");
  uint64_t cur = pos;
  for (uint32_t i = 0; i < size; ++i) {
    RoaringContainer c{};
    c.key = le16(desc + 4 * i);
    const uint32_t card = (uint32_t)le16(desc + 4 * i + 2) + 1;
    const bool is_run = run_flags && ((run_flags[i / 8] >> (i % 8)) & 1);
    uint64_t at = has_offsets ? le32(offs + 4 * i) : cur;
    uint64_t bytes;
    if (is_run) {
      c.type = 2;
      if (at + 2 > len) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated run container");
      c.card = le16(blob + at);
      bytes = 2 + 4ull * c.card;
    } else if (card <= 4096) {
      c.type = 0;
      c.card = (int32_t)card;
      bytes = 2ull * card;
    } else {
      c.type = 1;
      c.card = (int32_t)card;
      bytes = 8192;
    }
    if (at + bytes > len) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated container");
    c.offset = blob_offset + at;
    cur = at + bytes;
    out.push_back(c);
  }
}

void collect_bitmap_containers(const Column& c, const std::vector<int32_t>& ids, std::vector<RoaringContainer>& out) {
  // BitmapInvertedIndexReader.getDocIds: offsets are uint32 BE; normalise by the first offset
  // (absolute or relative formats, BitmapInvertedIndexReader.java:40-61)
  const uint8_t* b = c.inverted.data();
  const uint64_t off_end = 4ull * (c.cardinality + 1);
  const uint64_t first = be32u(b);
  for (int32_t id : ids) {
    uint64_t s = be32u(b + 4ull * id) - first, e = be32u(b + 4ull * (id + 1)) - first;
    if (off_end + e > c.inverted.size() || e < s) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: bad offsets");
    parse_roaring(b + off_end + s, e - s, off_end + s, out);
  }
}

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
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    g->id = ctx->next_id++;
  }
  return g;
}

// dictId -> global id; nullptr when identity
const int32_t* segment_remap(Context* ctx, Column& c, const GlobalDict& g) {
  std::lock_guard<std::mutex> lk(c.cache_mu);
  auto it = c.remaps.find(g.id);
  if (it != c.remaps.end()) return it->second ? it->second->as<int32_t>() : nullptr;
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
    PH_HIP_CHECK(hipMemcpy(buf->ptr, map.data(), sizeof(int32_t) * map.size(), hipMemcpyHostToDevice));
  }
  c.remaps[g.id] = buf;
  return buf ? buf->as<int32_t>() : nullptr;
}

const uint32_t* segment_hll_table(Context* ctx, Column& c, int log2m) {
  std::lock_guard<std::mutex> lk(c.cache_mu);
  auto it = c.hll_tables.find(log2m);
  if (it != c.hll_tables.end()) return it->second.buf->as<uint32_t>();
  HllTable t;
  t.buf = std::make_unique<DeviceBuffer>();
  t.buf->alloc(sizeof(uint32_t) * std::max(1, c.cardinality), ctx->device);
  if (c.data_type == PH_STRING) {
    // MurmurHash.hash(String.getBytes()) = hash(bytes, len, -1)
    std::vector<uint32_t> h(c.cardinality);
    for (int32_t i = 0; i < c.cardinality; ++i) {
      const std::string& s = c.dict.strings[i];
      h[i] = hll_entry(murmur_hash_bytes(reinterpret_cast<const uint8_t*>(s.data()), (int32_t)s.size(), -1), log2m);
    }
    PH_HIP_CHECK(hipMemcpy(t.buf->ptr, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice));
  } else if (c.data_type == PH_FLOAT) {
    fail(PH_ERR_UNSUPPORTED, "DISTINCTCOUNTHLL on FLOAT columns is not on the GPU path");
  } else {
    // INT / LONG -> hashLong((long) value); DOUBLE -> hashLong(doubleToRawLongBits)
    launch_hll_table(c.d_values.ptr, c.data_type != PH_DOUBLE, c.cardinality, log2m, t.buf->as<uint32_t>(),
                     ctx->stream);
    PH_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  }
  const uint32_t* p = t.buf->as<uint32_t>();
  c.hll_tables[log2m] = std::move(t);
  return p;
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
struct QueryScratch {
  std::vector<std::unique_ptr<DeviceBuffer>> bufs;
  int device;
  explicit QueryScratch(int d) : device(d) {}
  template <class T>
  T* alloc(size_t count) {
    auto b = std::make_unique<DeviceBuffer>();
    b->alloc(std::max<size_t>(16, sizeof(T) * count), device);
    T* p = b->as<T>();
    bufs.push_back(std::move(b));
    return p;
  }
};

ph_result* query_execute_impl(Context* ctx, const ph_query* q, ph_segment* const* segs_in, int32_t nseg) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  if (!q) fail(PH_ERR_INVALID_ARGUMENT, "null query");
  if (nseg < 0 || (nseg > 0 && !segs_in)) fail(PH_ERR_INVALID_ARGUMENT, "bad segment list");
  if (q->num_aggregations > kMaxAggs) fail(PH_ERR_UNSUPPORTED, "too many aggregations");
  if (q->num_group_by > kMaxGroupCols) fail(PH_ERR_UNSUPPORTED, "too many group-by columns");
  std::lock_guard<std::mutex> qlock(ctx->mu);
  PH_HIP_CHECK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  std::vector<ph_segment*> segs(segs_in, segs_in + nseg);
  for (auto* s : segs)
    if (!s || s->ctx != ctx) fail(PH_ERR_INVALID_ARGUMENT, "segment is null or pinned on another context");

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
  int log2m = 0, num_hll = 0;
  std::vector<int> agg_hll(q->num_aggregations, -1);
  std::set<std::string> projected(group_cols.begin(), group_cols.end());
  for (int k = 0; k < q->num_aggregations; ++k) {
    const ph_aggregation& a = q->aggregations[k];
    res->agg_types.push_back(a.type);
    int lm = a.type == PH_AGG_DISTINCTCOUNTHLL ? (a.log2m > 0 ? a.log2m : 8) : 0;
    res->agg_log2m.push_back(lm);
    if (a.type < PH_AGG_COUNT || a.type > PH_AGG_DISTINCTCOUNTHLL) fail(PH_ERR_UNSUPPORTED, "aggregation type");
    if (a.type == PH_AGG_COUNT) continue;
    if (!a.column) fail(PH_ERR_BAD_QUERY, "aggregation needs a column");
    add_slot(a.column);
    projected.insert(a.column);
    if (a.type == PH_AGG_DISTINCTCOUNTHLL) {
      if (lm < 4 || lm > 16) fail(PH_ERR_UNSUPPORTED, "log2m out of range");
      if (log2m && lm != log2m) fail(PH_ERR_UNSUPPORTED, "DISTINCTCOUNTHLL with different log2m in one query");
      log2m = lm;
      agg_hll[k] = num_hll++;
    }
  }
  if (q->filter_root >= 0)
    for (int i = 0; i < q->num_predicates; ++i) {
      if (!q->predicates[i].column) fail(PH_ERR_BAD_QUERY, "predicate without column");
      add_slot(q->predicates[i].column);
    }
  if ((int)slot_names.size() > kMaxCols) fail(PH_ERR_UNSUPPORTED, "too many columns in one query");
  for (auto* s : segs)
    for (auto& c : slot_names) {
      auto it = s->columns.find(c);
      if (it == s->columns.end()) fail(PH_ERR_BAD_QUERY, "Column not found: " + c + " in segment " + s->name);
      for (int k = 0; k < q->num_aggregations; ++k) {
        const ph_aggregation& a = q->aggregations[k];
        if (a.column && c == a.column && (a.type == PH_AGG_SUM || a.type == PH_AGG_MIN || a.type == PH_AGG_MAX) &&
            it->second->data_type == PH_STRING)
          fail(PH_ERR_UNSUPPORTED, "numeric aggregation on STRING column " + c);
      }
    }
  const int nagg = q->num_aggregations;
  const int m = log2m ? (1 << log2m) : 0;

  // ---- aggregation-only, no filter, metadata-answerable (NonScanBasedAggregationOperator)
  bool non_scan = q->filter_root < 0 && q->num_group_by == 0 && nagg > 0;
  for (int k = 0; k < nagg && non_scan; ++k) non_scan = q->aggregations[k].type != PH_AGG_SUM;
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
          const uint32_t* dt = segment_hll_table(ctx, c, lm);
          std::vector<uint32_t> h(c.cardinality);
          PH_HIP_CHECK(hipMemcpy(h.data(), dt, sizeof(uint32_t) * h.size(), hipMemcpyDeviceToHost));
          for (uint32_t e : h) regs[e >> 8] = std::max<uint8_t>(regs[e >> 8], (uint8_t)(e & 0xff));
        }
      }
    }
    stats.num_docs_scanned = stats.num_total_docs;
    stats.num_segments_matched = nseg;
    stats.host_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    return res.release();
  }

  // ---- per-segment filter plans
  QueryScratch scratch(ctx->device);
  std::vector<SegProgram> progs(nseg);
  std::vector<char> seg_live(nseg, 1);
  std::vector<int> seg_fast(nseg, 0);
  for (int i = 0; i < nseg; ++i) {
    PNode root;
    root.kind = L_ALL;
    if (q->filter_root >= 0) root = pl.build(segs[i], q->filter_root, 0);
    stats.num_entries_scanned_in_filter += (int64_t)segs[i]->num_docs * count_scan_leaves(root);
    if (root.kind == L_NONE || segs[i]->num_docs == 0) {
      seg_live[i] = 0;
      continue;
    }
    if (root.kind == L_ALL) {
      seg_fast[i] = 2;
      continue;
    }
    if (root.op == OP_RANGE) seg_fast[i] = 1;
    emit(root, progs[i]);
    if (progs[i].max_depth > kMaxStack || (int)progs[i].insns.size() > kMaxProg)
      fail(PH_ERR_UNSUPPORTED, "filter too large for the GPU program");
    for (auto& in : progs[i].insns)
      if ((in.op == OP_AND || in.op == OP_OR) && in.col > kMaxStack) fail(PH_ERR_UNSUPPORTED, "filter too wide");
  }

  // ---- inverted-index leaves -> device doc bitmaps
  for (auto& b : pl.bitmaps) {
    (void)b;
  }
  std::vector<uint32_t*> bitmap_dev(pl.bitmaps.size(), nullptr);
  for (size_t i = 0; i < pl.bitmaps.size(); ++i) {
    BitmapLeaf& b = pl.bitmaps[i];
    const size_t words = ((size_t)b.seg->num_docs + 31) / 32 + 1;
    uint32_t* bm = scratch.alloc<uint32_t>(words);
    PH_HIP_CHECK(hipMemsetAsync(bm, 0, words * 4, st));
    std::vector<RoaringContainer> cs;
    collect_bitmap_containers(*b.col, b.dict_ids, cs);
    if (!cs.empty()) {
      RoaringContainer* dc = scratch.alloc<RoaringContainer>(cs.size());
      PH_HIP_CHECK(hipMemcpyAsync(dc, cs.data(), sizeof(RoaringContainer) * cs.size(), hipMemcpyHostToDevice, st));
      launch_roaring_or(dc, (int)cs.size(), b.col->d_inverted.as<uint8_t>(), bm, b.seg->num_docs, st);
    }
    bitmap_dev[i] = bm;
    PH_HIP_CHECK(hipStreamSynchronize(st));  // `cs` is pageable host memory
  }

  // ---- group-by key space over table-level dictionaries
  std::vector<std::shared_ptr<GlobalDict>> gdicts;
  int64_t num_groups = 1;
  for (auto& g : group_cols) {
    std::shared_ptr<GlobalDict> gd;
    auto it = ctx->table_dicts.find(g);
    if (it != ctx->table_dicts.end()) {
      gd = it->second;
    } else {
      std::string key = g + "#";
      for (auto* s : segs) key += std::to_string(s->id) + ",";
      auto ct = ctx->union_cache.find(key);
      if (ct != ctx->union_cache.end()) {
        gd = ct->second;
      } else {
        gd = build_union(ctx, g, segs);
        if (ctx->union_cache.size() > 256) ctx->union_cache.clear();
        ctx->union_cache[key] = gd;
      }
    }
    gdicts.push_back(gd);
    if (gd->dict.size <= 0) gd->dict.size = 1;
    if (num_groups > (int64_t(1) << 40) / gd->dict.size) fail(PH_ERR_UNSUPPORTED, "group key space too large");
    num_groups *= gd->dict.size;
  }
  // numGroupsLimit: segments whose key space exceeds the limit may drop groups in the reference
  // (first-seen order, IntGroupIdMap.getGroupId :992-1017); that emulation is not on the GPU path.
  if (q->num_group_by > 0) {
    const int64_t limit = q->num_groups_limit > 0 ? q->num_groups_limit : 100000;
    for (auto* s : segs) {
      int64_t p = 1;
      for (auto& g : group_cols) p = std::min<int64_t>(p * s->columns.at(g)->cardinality, int64_t(1) << 40);
      if (p > limit)
        fail(PH_ERR_UNSUPPORTED, "segment " + s->name + ": product of group-by cardinalities " + std::to_string(p) +
                                     " exceeds numGroupsLimit " + std::to_string(limit));
    }
  }

  // ---- mode selection
  int mode;
  size_t lds = 0;
  KParams kp{};
  kp.num_aggs = nagg;
  kp.num_hll = num_hll;
  kp.log2m = log2m ? log2m : 8;
  kp.num_groups = num_groups;
  kp.num_group_cols = q->num_group_by;
  for (int g = 0, stride = 1; g < q->num_group_by; ++g) (void)stride;
  {
    int64_t stride = 1;
    for (int g = 0; g < q->num_group_by; ++g) {
      kp.group_slot[g] = pl.slot.at(group_cols[g]);
      kp.group_stride[g] = stride;
      stride *= gdicts[g]->dict.size;
    }
  }
  bool only_count = true;
  for (int k = 0; k < nagg; ++k) {
    const ph_aggregation& a = q->aggregations[k];
    kp.agg_type[k] = a.type;
    kp.agg_hll[k] = agg_hll[k] < 0 ? 0 : agg_hll[k];
    if (a.type != PH_AGG_COUNT) {
      only_count = false;
      kp.agg_slot[k] = pl.slot.at(a.column);
      const int dt = segs.empty() ? PH_INT : segs[0]->columns.at(a.column)->data_type;
      kp.agg_is_int[k] = (dt == PH_INT || dt == PH_LONG);
      for (auto* s : segs)
        if ((s->columns.at(a.column)->data_type == PH_INT || s->columns.at(a.column)->data_type == PH_LONG) !=
            (bool)kp.agg_is_int[k])
          fail(PH_ERR_UNSUPPORTED, "aggregation column with mixed integer/real types across segments");
    }
  }
  if (q->num_group_by == 0) {
    mode = only_count ? MODE_COUNT : MODE_AGG;
    lds = (size_t)num_hll * (m ? m : 1) * 4 + 16;
    kp.lds_hll_off = 0;
  } else {
    size_t off = ((size_t)num_groups * 4 + 15) / 16 * 16;
    for (int k = 0; k < nagg; ++k) {
      if (kp.agg_type[k] == AGG_COUNT || kp.agg_type[k] == AGG_HLL) continue;
      kp.lds_off[k] = (int32_t)std::min<size_t>(off, INT32_MAX);
      off += (size_t)num_groups * 8;
      off = (off + 15) / 16 * 16;
    }
    kp.lds_hll_off = (int32_t)std::min<size_t>(off, INT32_MAX);
    off += (size_t)num_groups * num_hll * (m ? m : 1) * 4;
    if (off <= 64 * 1024) {
      mode = MODE_GROUP_LDS;
      lds = off;
    } else {
      mode = MODE_GROUP_GLOBAL;
      lds = 16;
      const double bytes = (double)num_groups * (8 + 8.0 * nagg + 4.0 * num_hll * (m ? m : 1));
      if (bytes > 32e9) fail(PH_ERR_UNSUPPORTED, "dense group table too large for HBM budget");
    }
  }

  // ---- outputs
  const int64_t G = num_groups;
  kp.out_count = scratch.alloc<unsigned long long>(G);
  PH_HIP_CHECK(hipMemsetAsync(kp.out_count, 0, sizeof(unsigned long long) * G, st));
  for (int k = 0; k < nagg; ++k) {
    const int t = kp.agg_type[k];
    if (t == AGG_COUNT || t == AGG_HLL) continue;
    kp.out_agg[k] = scratch.alloc<int64_t>(G);
    if (t == AGG_SUM) PH_HIP_CHECK(hipMemsetAsync(kp.out_agg[k], 0, 8 * G, st));
    else launch_fill_i64((int64_t*)kp.out_agg[k], t == AGG_MIN ? INT64_MAX : INT64_MIN, G, st);
  }
  const int64_t hll_words = G * num_hll * (m ? m : 1);
  if (num_hll) {
    kp.out_hll = scratch.alloc<uint32_t>(hll_words);
    PH_HIP_CHECK(hipMemsetAsync(kp.out_hll, 0, 4 * hll_words, st));
  }

  // ---- device segment table, programs, chunks
  std::vector<DevSegment> dsegs;
  std::vector<FilterInsn> all_insns;
  std::vector<Chunk> chunks;
  constexpr int kChunkWords = 256;  // 16384 docs per chunk
  std::vector<std::pair<size_t, std::vector<uint32_t>>> payload_fix;  // global insn index -> payload
  std::vector<std::pair<size_t, int>> bitmap_fix;
  for (int i = 0; i < nseg; ++i) {
    if (!seg_live[i]) continue;
    ph_segment* s = segs[i];
    DevSegment d{};
    d.num_docs = s->num_docs;
    d.prog_off = (int32_t)all_insns.size();
    d.prog_len = (int32_t)progs[i].insns.size();
    d.fast_range = seg_fast[i];
    if (seg_fast[i] == 1) {
      d.fast_col = progs[i].insns[0].col;
      d.fast_lo = progs[i].insns[0].lo;
      d.fast_len = progs[i].insns[0].len;
    }
    for (auto& pp : progs[i].payloads) payload_fix.push_back({d.prog_off + pp.first, pp.second});
    for (auto& bb : progs[i].bitmap_refs) bitmap_fix.push_back({d.prog_off + bb.first, bb.second});
    all_insns.insert(all_insns.end(), progs[i].insns.begin(), progs[i].insns.end());
    for (size_t sl = 0; sl < slot_names.size(); ++sl) {
      Column& c = *s->columns.at(slot_names[sl]);
      DevColumn& dc = d.cols[sl];
      dc.fwd = c.d_fwd.as<uint32_t>();
      dc.bits = c.bits;
      dc.cardinality = c.cardinality;
      dc.values = c.d_values.ptr;
    }
    for (int g = 0; g < q->num_group_by; ++g)
      d.cols[kp.group_slot[g]].remap = segment_remap(ctx, *s->columns.at(group_cols[g]), *gdicts[g]);
    for (int k = 0; k < nagg; ++k)
      if (q->aggregations[k].type == PH_AGG_DISTINCTCOUNTHLL)
        d.cols[kp.agg_slot[k]].hll = segment_hll_table(ctx, *s->columns.at(q->aggregations[k].column), log2m);
    const int32_t words = (s->num_docs + 63) / 64;
    const int32_t seg_index = (int32_t)dsegs.size();
    for (int32_t w = 0; w < words; w += kChunkWords) chunks.push_back({seg_index, w, std::min(words, w + kChunkWords), 0});
    dsegs.push_back(d);
    stats.num_segments_matched++;
  }
  // payload buffers
  for (auto& pf : payload_fix) {
    uint32_t* dp = scratch.alloc<uint32_t>(pf.second.size() + 1);
    PH_HIP_CHECK(hipMemcpyAsync(dp, pf.second.data(), 4 * pf.second.size(), hipMemcpyHostToDevice, st));
    all_insns[pf.first].ptr = dp;
  }
  for (auto& bf : bitmap_fix) all_insns[bf.first].ptr = bitmap_dev[bf.second];

  float dev_ms = 0.f;
  if (!chunks.empty()) {
    DevSegment* d_segs = scratch.alloc<DevSegment>(dsegs.size());
    FilterInsn* d_prog = scratch.alloc<FilterInsn>(std::max<size_t>(1, all_insns.size()));
    Chunk* d_chunks = scratch.alloc<Chunk>(chunks.size());
    const size_t b1 = sizeof(DevSegment) * dsegs.size(), b2 = sizeof(FilterInsn) * all_insns.size(),
                 b3 = sizeof(Chunk) * chunks.size();
    uint8_t* stage = static_cast<uint8_t*>(ctx->host_staging(b1 + b2 + b3));
    memcpy(stage, dsegs.data(), b1);
    memcpy(stage + b1, all_insns.data(), b2);
    memcpy(stage + b1 + b2, chunks.data(), b3);
    PH_HIP_CHECK(hipMemcpyAsync(d_segs, stage, b1, hipMemcpyHostToDevice, st));
    if (b2) PH_HIP_CHECK(hipMemcpyAsync(d_prog, stage + b1, b2, hipMemcpyHostToDevice, st));
    PH_HIP_CHECK(hipMemcpyAsync(d_chunks, stage + b1 + b2, b3, hipMemcpyHostToDevice, st));
    kp.segs = d_segs;
    kp.prog = d_prog;
    kp.chunks = d_chunks;
    kp.num_chunks = (int32_t)chunks.size();
    kp.lds_bytes = (int32_t)lds;
    int blocks_per_cu = 8;
    if (mode == MODE_GROUP_LDS) blocks_per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
    const int grid = (int)std::min<int64_t>((int64_t)chunks.size(), (int64_t)ctx->num_cus * blocks_per_cu);
    PH_HIP_CHECK(hipEventRecord(ctx->ev_start, st));
    launch_scan(kp, mode, grid, 256, lds, st);
    PH_HIP_CHECK(hipEventRecord(ctx->ev_stop, st));
    PH_HIP_CHECK(hipStreamSynchronize(st));  // staging buffer reuse + results
    PH_HIP_CHECK(hipEventElapsedTime(&dev_ms, ctx->ev_start, ctx->ev_stop));
  } else {
    PH_HIP_CHECK(hipStreamSynchronize(st));
  }
  stats.device_ms = dev_ms;

  // ---- results
  int ncols_proj = (int)projected.size();
  if (q->num_group_by == 0) {
    init_row_results(1);
    unsigned long long matched = 0;
    PH_HIP_CHECK(hipMemcpy(&matched, kp.out_count, 8, hipMemcpyDeviceToHost));
    // segments whose filter matched everything (fast_range == 2) are scanned by the kernel as well
    stats.num_docs_scanned = (int64_t)matched;
    for (int k = 0; k < nagg; ++k) {
      const int t = kp.agg_type[k];
      uint8_t* dst = res->aggs[k].data();
      if (t == AGG_COUNT) {
        int64_t v = (int64_t)matched;
        memcpy(dst, &v, 8);
      } else if (t == AGG_HLL) {
        std::vector<uint32_t> r(m);
        PH_HIP_CHECK(hipMemcpy(r.data(), kp.out_hll + (size_t)agg_hll[k] * m, 4 * m, hipMemcpyDeviceToHost));
        for (int j = 0; j < m; ++j) dst[j] = (uint8_t)r[j];
      } else {
        int64_t raw;
        PH_HIP_CHECK(hipMemcpy(&raw, kp.out_agg[k], 8, hipMemcpyDeviceToHost));
        double v;
        if (t == AGG_SUM) {
          if (kp.agg_is_int[k]) {
            v = (double)raw;
            if (raw >= (int64_t(1) << 53) || raw <= -(int64_t(1) << 53)) stats.sum_precision_flag = 1;
          } else {
            memcpy(&v, &raw, 8);
          }
        } else if (matched == 0) {
          v = t == AGG_MIN ? INFINITY : -INFINITY;  // Min/MaxAggregationFunction defaults
        } else {
          v = kp.agg_is_int[k] ? (double)raw : double_from_order_key(raw);
        }
        memcpy(dst, &v, 8);
      }
    }
  } else {
    std::vector<unsigned long long> cnt(G);
    PH_HIP_CHECK(hipMemcpy(cnt.data(), kp.out_count, 8 * G, hipMemcpyDeviceToHost));
    std::vector<int64_t> live;
    for (int64_t g = 0; g < G; ++g)
      if (cnt[g]) {
        live.push_back(g);
        stats.num_docs_scanned += (int64_t)cnt[g];
      }
    const int64_t R = (int64_t)live.size();
    res->num_groups = R;
    init_row_results(R);
    std::vector<int64_t> buf;
    for (int k = 0; k < nagg; ++k) {
      const int t = kp.agg_type[k];
      uint8_t* dst = res->aggs[k].data();
      if (t == AGG_COUNT) {
        for (int64_t r = 0; r < R; ++r) {
          int64_t v = (int64_t)cnt[live[r]];
          memcpy(dst + 8 * r, &v, 8);
        }
      } else if (t == AGG_HLL) {
        std::vector<uint32_t> regs(hll_words);
        PH_HIP_CHECK(hipMemcpy(regs.data(), kp.out_hll, 4 * hll_words, hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < R; ++r)
          for (int j = 0; j < m; ++j) dst[(size_t)r * m + j] = (uint8_t)regs[((size_t)live[r] * num_hll + agg_hll[k]) * m + j];
      } else {
        buf.resize(G);
        PH_HIP_CHECK(hipMemcpy(buf.data(), kp.out_agg[k], 8 * G, hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < R; ++r) {
          const int64_t raw = buf[live[r]];
          double v;
          if (t == AGG_SUM) {
            if (kp.agg_is_int[k]) {
              v = (double)raw;
              if (raw >= (int64_t(1) << 53) || raw <= -(int64_t(1) << 53)) stats.sum_precision_flag = 1;
            } else {
              memcpy(&v, &raw, 8);
            }
          } else {
            v = kp.agg_is_int[k] ? (double)raw : double_from_order_key(raw);
          }
          memcpy(dst + 8 * r, &v, 8);
        }
      }
    }
    // keys
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
        const int64_t id = (live[r] / kp.group_stride[g]) % d.size;
        put_key_value(d, id, res->keys[g].data() + (size_t)es * r, es);
      }
    }
  }
  stats.num_entries_scanned_post_filter = stats.num_docs_scanned * ncols_proj;
  stats.host_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count() - dev_ms;
  return res.release();
}

}  // namespace ph
