// api.cpp -- extern "C" entry points of libpinot_hip.so (include/pinot_hip.h).  No C++ exception crosses
// the ABI: every entry point returns a PH_* status and leaves a thread-local message for ph_last_error().
#include <algorithm>
#include <cstring>
#include <new>

#include "ph_internal.h"

namespace ph {
thread_local std::string g_last_error;

const char* const kOptNames[OPT_COUNT] = {
    "roaring_atomic",
    "agg_cont",
    "group_cont",
    "disable_partition",
    "lds_table_max",
    "no_group_cache",
    "group_sparse",
    "agg_sparse",
    "tile_words",
    "limit_eager",
    "part_generic",
    "agg_generic",
    "lds_generic",
    "count_generic",
    "lds_lean",
    "group_reg_lg",
    "stat_fuse",
    "interrupt_chunks",
    "part_klo",
    "part_batch_rows",
    "part_flush_first",
    "part_depth",
    "part_lds",
    "part_sets",
    "part_wg_per_cu",
    "part_slices",
    "part_mm_blind",
    "part_serial",
    "part_ring_log2",
    "multi_host_merge",
    "sparse_c"
};

void fail(int code, const std::string& msg) { throw Error{code, msg}; }

ph_segment* segment_pin_impl(Context* ctx, const ph_segment_desc* desc);
ph_result* query_execute_impl(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg,
                              const DenseArgs* dense);
ph_result* segment_trim_execute(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg);  // trim.cpp
// multi.cpp
void context_init(Context& c, int ordinal);
void multi_init(ph_ctx* x, const int32_t* ordinals, int32_t n);
Context* place_segment(ph_ctx* x, int64_t rows);
void multi_set_transport(ph_ctx* x, int32_t transport);
ph_result* multi_execute(ph_ctx* x, const ph_query* q, ph_segment* const* segs, int32_t nseg);
}  // namespace ph

using namespace ph;

template <class F>
static int guarded(F&& f) {
  try {
    f();
    g_last_error.clear();
    return PH_OK;
  } catch (const Error& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host out of memory";
    return PH_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return PH_ERR_INVALID_ARGUMENT;
  } catch (...) {
    g_last_error = "unknown error";
    return PH_ERR_DEVICE;
  }
}

// a multi-device context pins on the device with the fewest docs (its rows reserved during the pin, which then
// counts them itself)
template <class F>
static ph_segment* pin_placed(ph_ctx* ctx, int64_t rows, F&& pin) {
  Context* c = place_segment(ctx, rows);
  const int64_t reserved = ctx->devs.size() > 1 ? rows : 0;
  ph_segment* s = nullptr;
  try {
    s = pin(c);
  } catch (...) {
    c->pinned_rows -= reserved;
    throw;
  }
  c->pinned_rows -= reserved;
  return s;
}

namespace ph {
// drops what the context cached for a segment: its remaps to table / union dictionaries and the unions that include
// it (never hit again: a re-pinned segment gets a new id)
void star_tree_forget(Context& c, ph_segment* seg) {
  std::lock_guard<std::mutex> lk(c.mu);
  for (auto& kv : c.table_dicts) {
    std::lock_guard<std::mutex> gl(kv.second->mu);
    kv.second->remaps.erase(seg->id);
  }
  const std::string tag = std::to_string(seg->id) + ",";
  auto holds = [&](const std::string& key) {
    const size_t h = key.find('#');
    for (size_t p = key.find(tag, h); p != std::string::npos; p = key.find(tag, p + 1))
      if (key[p - 1] == '#' || key[p - 1] == ',') return true;
    return false;
  };
  for (auto it = c.union_order.begin(); it != c.union_order.end();) {
    if (holds(*it)) {
      c.union_cache.erase(*it);
      it = c.union_order.erase(it);
    } else {
      ++it;
    }
  }
}
void star_tree_add_impl(ph_segment* seg, const ph_star_tree_desc* d);
void star_tree_check_impl(const void* tree, uint64_t size, int32_t* num_nodes, int32_t* num_dimensions);
}  // namespace ph

extern "C" {

const char* ph_last_error(void) { return g_last_error.c_str(); }
const char* ph_version(void) { return "pinot_hip 0.1.0 (gfx950)"; }

int ph_ctx_create(int32_t device_ordinal, ph_ctx** out) { return ph_ctx_create_multi(&device_ordinal, 1, out); }

int ph_ctx_create_multi(const int32_t* device_ordinals, int32_t num_devices, ph_ctx** out) {
  return guarded([&] {
    if (!out) fail(PH_ERR_INVALID_ARGUMENT, "out is null");
    auto* ctx = new ph_ctx();
    try {
      multi_init(ctx, device_ordinals, num_devices);
    } catch (...) {
      delete ctx;
      throw;
    }
    *out = ctx;
  });
}

int32_t ph_ctx_num_devices(const ph_ctx* ctx) { return ctx ? (int32_t)ctx->devs.size() : 0; }

int ph_ctx_set_multi_transport(ph_ctx* ctx, int32_t transport) {
  return guarded([&] {
    if (!ctx) fail(PH_ERR_INVALID_ARGUMENT, "ctx is null");
    multi_set_transport(ctx, transport);
  });
}

int ph_ctx_set_option(ph_ctx* ctx, const char* name, int64_t value) {
  return guarded([&] {
    if (!ctx || !name) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    for (int o = 0; o < OPT_COUNT; ++o)
      if (std::strcmp(kOptNames[o], name) == 0) {
        for (Context* c : ctx->devs) c->opts[o].store(value, std::memory_order_relaxed);
        return;
      }
    fail(PH_ERR_INVALID_ARGUMENT, std::string("unknown option ") + name);
  });
}

int ph_ctx_destroy(ph_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return;
    (void)hipSetDevice(ctx->c.device);
    delete ctx;  // Context::~Context drains and frees the lanes and the pinned pool
  });
}

int ph_ctx_set_stream(ph_ctx* ctx, void* hip_stream) {
  return guarded([&] {
    if (!ctx) fail(PH_ERR_INVALID_ARGUMENT, "ctx is null");
    if (ctx->devs.size() > 1) fail(PH_ERR_INVALID_ARGUMENT, "a multi-device context runs on its own streams");
    ctx->c.ext_stream.store(static_cast<hipStream_t>(hip_stream));
  });
}

int ph_segment_pin(ph_ctx* ctx, const ph_segment_desc* desc, ph_segment** out) {
  return guarded([&] {
    if (!ctx || !out) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    *out = pin_placed(ctx, desc ? desc->num_docs : 0, [&](Context* c) { return segment_pin_impl(c, desc); });
  });
}

int32_t ph_segment_device(const ph_segment* seg) { return seg && seg->ctx ? seg->ctx->device_index : -1; }

int ph_segment_load_dir(ph_ctx* ctx, const char* segment_dir, const char* const* columns, int32_t num_columns,
                        ph_segment** out) {
  return guarded([&] {
    if (!ctx || !out) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    // rows reserved from the metadata at placement, so concurrent loads (server start) spread over the devices
    *out = pin_placed(ctx, segment_dir_num_docs(segment_dir),
                      [&](Context* c) { return segment_load_dir_impl(c, segment_dir, columns, num_columns); });
  });
}

int ph_segment_check(const ph_segment_desc* desc) {
  return guarded([&] { segment_check_impl(desc); });
}


int ph_segment_unpin(ph_segment* seg) {
  return guarded([&] {
    if (!seg) return;
    (void)hipSetDevice(seg->ctx->device);
    ph::Context& c = *seg->ctx;
    ph::star_tree_forget(c, seg);  // (its star-tree views forget theirs as they are freed)
    c.pinned_rows -= seg->num_docs;
    delete seg;  // hipFree waits for work in flight on the buffers
  });
}

int ph_segment_add_star_tree(ph_segment* seg, const ph_star_tree_desc* desc) {
  return guarded([&] {
    if (!seg) fail(PH_ERR_INVALID_ARGUMENT, "null segment");
    PH_HIP_CHECK(hipSetDevice(seg->ctx->device));
    ph::star_tree_add_impl(seg, desc);
  });
}

int32_t ph_segment_num_star_trees(const ph_segment* seg) { return seg ? (int32_t)seg->star_trees.size() : -1; }

int ph_star_tree_check(const void* tree, uint64_t tree_size, int32_t* num_nodes, int32_t* num_dimensions) {
  return guarded([&] { ph::star_tree_check_impl(tree, tree_size, num_nodes, num_dimensions); });
}

int64_t ph_segment_device_bytes(const ph_segment* seg) {
  if (!seg) return -1;
  int64_t n = seg->device_bytes;  // pinned columns, plus the caches queries built for them
  for (auto& kv : seg->columns) {
    ph::Column& c = *kv.second;
    std::lock_guard<std::mutex> lk(c.cache_mu);
    for (auto& h : c.hll_tables) n += h.second.buf ? (int64_t)h.second.buf->bytes : 0;
    if (c.d_vpacked) n += (int64_t)c.d_vpacked->bytes;
  }
  ph::Context& c = *seg->ctx;  // remaps to table / union dictionaries
  std::lock_guard<std::mutex> lk(c.mu);
  auto add = [&](ph::GlobalDict& g) {
    std::lock_guard<std::mutex> gl(g.mu);
    auto it = g.remaps.find(seg->id);
    if (it != g.remaps.end() && it->second) n += (int64_t)it->second->bytes;
  };
  for (auto& kv : c.table_dicts) add(*kv.second);
  for (auto& kv : c.union_cache) add(*kv.second);
  return n;
}
int32_t ph_segment_num_docs(const ph_segment* seg) { return seg ? seg->num_docs : -1; }

int ph_table_set_dictionary(ph_ctx* ctx, const char* column, int32_t data_type, const void* values, int64_t count,
                            int32_t entry_size) {
  return guarded([&] {
    if (!ctx || !column || (count > 0 && !values)) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    auto g = std::make_shared<GlobalDict>();
    Dictionary& d = g->dict;
    d.type = data_type;
    d.size = count;
    const uint8_t* b = static_cast<const uint8_t*>(values);
    switch (data_type) {
      case PH_INT:
        d.ints.resize(count);
        for (int64_t i = 0; i < count; ++i) d.ints[i] = reinterpret_cast<const int32_t*>(b)[i];
        break;
      case PH_LONG:
        d.ints.assign(reinterpret_cast<const int64_t*>(b), reinterpret_cast<const int64_t*>(b) + count);
        break;
      case PH_FLOAT:
        d.reals.resize(count);
        for (int64_t i = 0; i < count; ++i) d.reals[i] = reinterpret_cast<const float*>(b)[i];
        break;
      case PH_DOUBLE:
        d.reals.assign(reinterpret_cast<const double*>(b), reinterpret_cast<const double*>(b) + count);
        break;
      case PH_STRING:
        if (entry_size <= 0) fail(PH_ERR_INVALID_ARGUMENT, "entry_size");
        d.strings.resize(count);
        for (int64_t i = 0; i < count; ++i) {
          const char* s = reinterpret_cast<const char*>(b + (size_t)entry_size * i);
          d.strings[i].assign(s, strnlen(s, entry_size));
          d.max_string_len = std::max<int32_t>(d.max_string_len, (int32_t)d.strings[i].size());
        }
        break;
      default:
        fail(PH_ERR_INVALID_ARGUMENT, "data type");
    }
    for (int64_t i = 1; i < count; ++i)
      if (d.compare(i - 1, d, i) >= 0) fail(PH_ERR_INVALID_ARGUMENT, "table dictionary must be sorted and unique");
    for (Context* c : ctx->devs) {  // one copy per device: its device-side caches (values, remaps) live there
      auto gc = std::make_shared<GlobalDict>();
      gc->dict = g->dict;
      gc->id = next_object_id();
      std::lock_guard<std::mutex> lk(c->mu);
      c->table_dicts[column] = gc;
    }
  });
}

int ph_table_set_column_type(ph_ctx* ctx, const char* column, int32_t data_type) {
  return guarded([&] {
    if (!ctx || !column) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    if (data_type < PH_INT || data_type > PH_STRING) fail(PH_ERR_INVALID_ARGUMENT, "data type");
    for (Context* c : ctx->devs) {
      std::lock_guard<std::mutex> lk(c->mu);
      c->column_types[column] = data_type;
    }
  });
}

int ph_query_execute(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                     ph_result** out) {
  return guarded([&] {
    if (!ctx || !out) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (ctx->devs.size() > 1)
      *out = multi_execute(ctx, query, segments, num_segments);  // per device, merged in the library
    else if (query && query->min_segment_group_trim_size > 0 && query->num_group_by > 0 && query->num_order_by > 0)
      *out = segment_trim_execute(&ctx->c, query, segments, num_segments);  // GroupByOperator segment trim
    else
      *out = query_execute_impl(&ctx->c, query, segments, num_segments, nullptr);
  });
}

// Segment-level drop-in (FilterPlanNode.run -> BaseFilterOperator): one segment's filter as a COUNT(*) whose MODE_COUNT
// scan also writes the doc bitmap (DenseArgs::docset), the statistic computed exactly as for a query
int ph_filter_execute(ph_ctx* ctx, const ph_query* query, ph_segment* segment, uint64_t* doc_words, uint64_t num_words,
                      ph_exec_stats* stats) {
  return guarded([&] {
    if (!ctx || !query || !segment) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    Context* c = segment->ctx;
    bool mine = false;
    for (Context* d : ctx->devs) mine = mine || d == c;
    if (!mine) fail(PH_ERR_INVALID_ARGUMENT, "segment is pinned on another context");
    const int64_t nd = segment->num_docs;
    const uint64_t need = (uint64_t)((nd + 63) / 64);
    if (doc_words && num_words < need) fail(PH_ERR_INVALID_ARGUMENT, "doc_words holds fewer than ceil(num_docs / 64) words");
    ph_exec_stats st{};
    st.num_total_docs = nd;
    st.num_segments_processed = 1;
    if (query->filter_root < 0) {  // no WHERE clause: MatchAllFilterOperator (FilterPlanNode.java:96-101)
      if (doc_words) {
        for (uint64_t w = 0; w < need; ++w) doc_words[w] = ~0ull;
        if (nd % 64) doc_words[need - 1] = (1ull << (nd % 64)) - 1ull;
      }
      st.num_docs_scanned = nd;
      st.num_segments_matched = nd > 0;
      st.plan_mode = -2;
      if (stats) *stats = st;
      return;
    }
    // the filter as a COUNT(*) with no group-by, ordering or trim
    ph_query q = *query;
    ph_aggregation cnt{};
    cnt.type = PH_AGG_COUNT;
    q.num_group_by = 0;
    q.group_by = nullptr;
    q.num_aggregations = 1;
    q.aggregations = &cnt;
    q.num_order_by = 0;
    q.order_by = nullptr;
    q.min_segment_group_trim_size = -1;
    q.skip_star_tree = 1;  // FilterPlanNode's operator is over the segment's own documents
    ph_segment* segs[1] = {segment};
    std::unique_ptr<ph_result> r;
    if (!doc_words) {
      r.reset(query_execute_impl(c, &q, segs, 1, nullptr));
    } else {
      PH_HIP_CHECK(hipSetDevice(c->device));
      std::unique_ptr<DeviceBuffer> words = c->scratch_acquire(std::max<uint64_t>(1, need) * 8);
      struct Back {  // the scratch block goes back to the pool on every exit
        Context* c;
        std::unique_ptr<DeviceBuffer>& b;
        ~Back() { c->scratch_release(std::move(b)); }
      } back{c, words};
      const int64_t off[1] = {0};
      FilterDocset fd{words->as<unsigned long long>(), off, (int64_t)need};
      DenseArgs d{0, nullptr, 0, 0, nullptr};
      d.docset = &fd;
      r.reset(query_execute_impl(c, &q, segs, 1, &d));
      // the call drained its stream before it read the count
      if (need) PH_HIP_CHECK(hipMemcpy(doc_words, words->ptr, 8 * need, hipMemcpyDeviceToHost));
    }
    if (stats) *stats = r->stats;
  });
}

// Dense partials merge whole per-device tables, so GroupByOperator's per-segment trim (ORDER BY +
// minSegmentGroupTrimSize > 0, GroupByOperator.java:114-130) cannot apply: such queries are not served here (the caller
// takes ph_query_execute, which trims, or the CPU plan).
// the device context a dense call runs on: the one every segment is pinned on
static Context* dense_device(ph_ctx* ctx, ph_segment* const* segs, int32_t n) {
  Context* c = n > 0 && segs && segs[0] ? segs[0]->ctx : &ctx->c;
  for (int32_t i = 0; i < n; ++i)
    if (!segs[i] || segs[i]->ctx != c) fail(PH_ERR_INVALID_ARGUMENT, "dense partials take the segments of one device");
  return c;
}

static void reject_segment_trim(const ph_query* q) {
  if (q && q->min_segment_group_trim_size > 0 && q->num_group_by > 0 && q->num_order_by > 0)
    fail(PH_ERR_UNSUPPORTED, "segment group trim (minSegmentGroupTrimSize) on dense partials");
}

int ph_query_dense_layout(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                          ph_dense_layout* out) {
  return guarded([&] {
    if (!ctx || !out) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    reject_segment_trim(query);
    DenseArgs d{DENSE_LAYOUT, nullptr, 0, 0, out};
    query_execute_impl(dense_device(ctx, segments, num_segments), query, segments, num_segments, &d);
  });
}

int ph_query_execute_dense(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                           void* const* device_tables, ph_exec_stats* stats) {
  return guarded([&] {
    if (!ctx || !device_tables) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    reject_segment_trim(query);
    DenseArgs d{DENSE_EXECUTE, device_tables, 0, 0, nullptr};
    std::unique_ptr<ph_result> r(query_execute_impl(dense_device(ctx, segments, num_segments), query, segments,
                                                    num_segments, &d));
    if (stats && r) *stats = r->stats;
  });
}

int ph_dense_finalize(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                      const void* const* device_tables, int64_t group_begin, int64_t group_end, ph_result** out) {
  return guarded([&] {
    if (!ctx || !device_tables || !out) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    reject_segment_trim(query);
    DenseArgs d{DENSE_FINALIZE, const_cast<void* const*>(device_tables), group_begin, group_end, nullptr};
    *out = query_execute_impl(dense_device(ctx, segments, num_segments), query, segments, num_segments, &d);
  });
}

int ph_result_destroy(ph_result* r) {
  delete r;
  return PH_OK;
}

int ph_result_stats(const ph_result* r, ph_exec_stats* out) {
  return guarded([&] {
    if (!r || !out) fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    *out = r->stats;
  });
}

int64_t ph_result_num_groups(const ph_result* r) { return r ? r->num_groups : -1; }

int ph_result_key_entry_size(const ph_result* r, int32_t i) {
  if (!r || i < 0 || i >= (int32_t)r->key_entry_size.size()) return -1;
  return r->key_entry_size[i];
}

int ph_result_key_type(const ph_result* r, int32_t i) {
  if (!r || i < 0 || i >= (int32_t)r->key_types.size()) return -1;
  return r->key_types[i];
}

const void* ph_result_key_data(const ph_result* r, int32_t i) {
  if (!r || i < 0 || i >= (int32_t)r->keys.size()) return nullptr;
  return r->keys[i].data();
}

const void* ph_result_aggregation_data(const ph_result* r, int32_t k) {
  if (!r || k < 0 || k >= (int32_t)r->aggs.size()) return nullptr;
  return r->aggs[k].data();
}

int ph_result_group_keys(const ph_result* r, int32_t i, void* out) {
  return guarded([&] {
    if (!r || !out || i < 0 || i >= (int32_t)r->keys.size()) fail(PH_ERR_INVALID_ARGUMENT, "bad key index");
    memcpy(out, r->keys[i].data(), r->keys[i].size());
  });
}

int ph_result_aggregation(const ph_result* r, int32_t k, void* out) {
  return guarded([&] {
    if (!r || !out || k < 0 || k >= (int32_t)r->aggs.size()) fail(PH_ERR_INVALID_ARGUMENT, "bad aggregation index");
    memcpy(out, r->aggs[k].data(), r->aggs[k].size());
  });
}

int ph_selftest_unpack(ph_ctx* ctx, const uint8_t* packed, uint64_t packed_size, int64_t n, int32_t bits,
                       int32_t* out) {
  return guarded([&] {
    if (!ctx || !packed || !out || n < 0 || bits < 1 || bits > 31) fail(PH_ERR_INVALID_ARGUMENT, "bad arguments");
    if (packed_size < (uint64_t)((n * bits + 7) / 8)) fail(PH_ERR_INVALID_ARGUMENT, "packed buffer too small");
    PH_HIP_CHECK(hipSetDevice(ctx->c.device));
    LaneGuard lg(&ctx->c);
    const hipStream_t st = lg.lane->stream;
    DeviceBuffer in, o;
    in.alloc(packed_size + kFwdPadBytes, ctx->c.device);
    o.alloc(sizeof(int32_t) * std::max<int64_t>(1, n), ctx->c.device);
    PH_HIP_CHECK(hipMemsetAsync(in.ptr, 0, packed_size + kFwdPadBytes, st));
    PH_HIP_CHECK(hipMemcpyAsync(in.ptr, packed, packed_size, hipMemcpyHostToDevice, st));
    launch_selftest_unpack(in.as<uint32_t>(), n, bits, o.as<int32_t>(), st);
    PH_HIP_CHECK(hipMemcpyAsync(out, o.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
    PH_HIP_CHECK(hipStreamSynchronize(st));
  });
}

int ph_selftest_unpack_staged(ph_ctx* ctx, const uint8_t* packed, uint64_t packed_size, int64_t n, int32_t bits,
                              int32_t tile_words, int32_t* out) {
  return guarded([&] {
    if (!ctx || !packed || !out || n < 0 || n > INT32_MAX || bits < 1 || bits > 31)
      fail(PH_ERR_INVALID_ARGUMENT, "bad arguments");
    if (tile_words < 1 || tile_words > kMaxTileWords) fail(PH_ERR_INVALID_ARGUMENT, "tile_words out of range");
    if (packed_size < (uint64_t)((n * bits + 7) / 8)) fail(PH_ERR_INVALID_ARGUMENT, "packed buffer too small");
    if (stage_loads(tile_words, bits) > kPrefetchOther) fail(PH_ERR_UNSUPPORTED, "tile too wide for the prefetch pool");
    PH_HIP_CHECK(hipSetDevice(ctx->c.device));
    LaneGuard lg(&ctx->c);
    const hipStream_t st = lg.lane->stream;
    DeviceBuffer in, o, dseg;
    in.alloc(packed_size + kFwdPadBytes, ctx->c.device);
    o.alloc(sizeof(int32_t) * std::max<int64_t>(1, n), ctx->c.device);
    dseg.alloc(sizeof(DevSegment), ctx->c.device);
    PH_HIP_CHECK(hipMemsetAsync(in.ptr, 0, packed_size + kFwdPadBytes, st));
    PH_HIP_CHECK(hipMemcpyAsync(in.ptr, packed, packed_size, hipMemcpyHostToDevice, st));
    DevSegment d{};
    d.num_docs = (int32_t)n;
    d.streams[0] = DevStream{in.as<uint32_t>(), bits, 0};
    const int32_t soff[1] = {0};
    fill_tile_pieces(d, 1, soff, tile_words);
    PH_HIP_CHECK(hipMemcpyAsync(dseg.ptr, &d, sizeof(d), hipMemcpyHostToDevice, st));
    const int32_t stride = stage_stream_bytes(tile_words, bits);
    launch_selftest_staged(dseg.as<DevSegment>(), tile_words, stride, n, o.as<int32_t>(), st);
    PH_HIP_CHECK(hipMemcpyAsync(out, o.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
    PH_HIP_CHECK(hipStreamSynchronize(st));
  });
}

int ph_result_datatable(const ph_result* r, const ph_query* q, const ph_metadata_entry* extra, int32_t num_extra,
                        void* out, uint64_t capacity, uint64_t* size) {
  return guarded([&] {
    if (!size || num_extra < 0 || (num_extra > 0 && !extra)) ph::fail(PH_ERR_INVALID_ARGUMENT, "bad arguments");
    const auto bytes = ph::result_to_datatable(r, q, extra, num_extra);
    *size = bytes.size();
    if (out) {
      if (capacity < bytes.size()) ph::fail(PH_ERR_INVALID_ARGUMENT, "DataTable buffer too small");
      memcpy(out, bytes.data(), bytes.size());
    }
  });
}

int ph_raw_forward_index_read(const void* buf, uint64_t size, int32_t data_type, int32_t num_docs, void* out) {
  return guarded([&] {
    if (!buf || !out || num_docs < 0) ph::fail(PH_ERR_INVALID_ARGUMENT, "null buffer or negative num_docs");
    ph::raw_forward_index_decode(static_cast<const uint8_t*>(buf), size, data_type, num_docs, out);
  });
}

int ph_index_map_lookup(const char* index_map_path, const char* column, const char* index_id, int64_t* start_offset,
                        int64_t* size) {
  return guarded([&] {
    if (!index_map_path || !column || !index_id || !start_offset || !size)
      ph::fail(PH_ERR_INVALID_ARGUMENT, "null argument");
    const ph::IndexMap m = ph::read_index_map(index_map_path);
    auto it = m.find({column, index_id});
    if (it == m.end()) ph::fail(PH_ERR_BAD_QUERY, std::string("index_map has no ") + column + "." + index_id);
    *start_offset = it->second.first;
    *size = it->second.second;
  });
}

int ph_fixed_bit_pack(const int32_t* dict_ids, int64_t n, int32_t bits, uint8_t* out, uint64_t out_size) {
  return guarded([&] {
    if (n < 0 || bits < 1 || bits > 31 || (n > 0 && (!dict_ids || !out)))
      fail(PH_ERR_INVALID_ARGUMENT, "bad pack arguments");
    const uint64_t need = (uint64_t)((n * bits + 7) / 8);
    if (out_size < need) fail(PH_ERR_INVALID_ARGUMENT, "output buffer too small");
    fixed_bit_pack_host(dict_ids, n, bits, out);
  });
}

}  // extern "C"
