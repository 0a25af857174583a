// multi.cpp -- one ph_ctx over several GPUs of a node (ph_ctx_create_multi): segment placement and the combine of the
// devices' partial results inside the library.
//
// A Pinot server runs every segment of a query in one JVM and merges their results in GroupByCombineOperator
// (GroupByCombineOperator.java:125-197: the per-segment tasks, then IndexedTable upserts keyed by group values).  Here
// the server's context owns one Context per GPU:
//  * ph_segment_pin places a segment on the device with the fewest pinned docs (greedy row balance);
//  * ph_query_execute splits the query's segments by device, scans each device's share into DENSE partial tables
//    over one set of table-level dictionaries (ph_query_execute_dense's tables: a group is the same dense id on
//    every device), one host thread per device, and merges the tables:
//      - distinct devices: RCCL reduce-scatter over xGMI (ncclCommInitAll, in-process; librccl is dlopen'ed), so
//        device k owns the fully merged key shard k and finalises it (ph_dense_finalize's compaction) in parallel
//        with the others; the shards concatenate into one ph_result;
//      - logical shards sharing a device (e.g. a test of two shards on one GPU): a device copy + reduce kernel into
//        the first shard's tables, finalised whole;
//  * a query the dense tables do not serve (a key space beyond the dense budget, group trim) runs per device and
//    the per-device results merge on the host by group value (merge_results_by_value).
#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <exception>
#include <map>
#include <thread>

#include <rccl/rccl.h>

#include "host_pool.h"
#include "ph_internal.h"

namespace ph {

ph_result* query_execute_impl(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg,
                              const DenseArgs* dense);
ph_result* segment_trim_execute(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg);

namespace {

// librccl.so.1 entry points, loaded on first use (RTLD_LOCAL: no link-time dependency, and no clash with another RCCL
// already in the process, such as torch's)
struct Rccl {
  void* h = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    x.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!x.h) x.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!x.h) return x;
    x.init_all = reinterpret_cast<decltype(x.init_all)>(dlsym(x.h, "ncclCommInitAll"));
    x.reduce_scatter = reinterpret_cast<decltype(x.reduce_scatter)>(dlsym(x.h, "ncclReduceScatter"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(dlsym(x.h, "ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(dlsym(x.h, "ncclGroupEnd"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(x.h, "ncclCommDestroy"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(x.h, "ncclGetErrorString"));
    if (!x.init_all || !x.reduce_scatter || !x.group_start || !x.group_end || !x.destroy || !x.error_string) x.h = nullptr;
    return x;
  }();
  if (!r.h) fail(PH_ERR_UNSUPPORTED, "librccl.so.1 is not loadable: the multi-GPU combine needs RCCL");
  return r;
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) fail(PH_ERR_DEVICE, std::string(what) + ": " + rccl().error_string(e));
}

ncclDataType_t nccl_type(int op) {
  return op == PH_REDUCE_SUM_F64 ? ncclFloat64 : (op == PH_REDUCE_MAX_U32 ? ncclUint32 : ncclInt64);
}
ncclRedOp_t nccl_op(int op) {
  return op == PH_REDUCE_MIN_I64 ? ncclMin : ((op == PH_REDUCE_MAX_I64 || op == PH_REDUCE_MAX_U32) ? ncclMax : ncclSum);
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

constexpr size_t kLayoutCacheEntries = 64;

// A device scratch block of one call, back to its context's pool when the call ends (after a throw, only once the
// device is idle: a collective or copy may still write it)
struct ScratchHold {
  Context* c = nullptr;
  std::unique_ptr<DeviceBuffer> b;
  ScratchHold() = default;
  ScratchHold(Context* ctx, size_t n) : c(ctx), b(ctx->scratch_acquire(n)) {}
  ScratchHold(ScratchHold&&) = default;
  ScratchHold& operator=(ScratchHold&&) = default;
  ~ScratchHold() {
    if (!b) return;
    if (std::uncaught_exceptions() > 0) {
      (void)hipSetDevice(c->device);
      (void)hipDeviceSynchronize();
    }
    c->scratch_release(std::move(b));
  }
  void* ptr() const { return b->ptr; }
};

// the layout cache key: what ph_query_dense_layout's answer depends on -- the group-by columns and aggregations, the
// segments (their column types and dictionaries), and the table dictionaries in force (their ids change when replaced)
std::string layout_key(ph_ctx* x, const ph_query* q, const std::vector<ph_segment*>& all) {
  std::string k;
  auto add = [&](const char* s) {
    k += s ? s : "\x01";
    k += '\0';
  };
  for (int g = 0; g < q->num_group_by; ++g) {
    add(q->group_by[g]);
    for (Context* c : x->devs) {
      std::lock_guard<std::mutex> lk(c->mu);
      auto it = c->table_dicts.find(q->group_by[g]);
      k += std::to_string(it == c->table_dicts.end() ? 0 : it->second->id) + ",";
    }
  }
  k += "|";
  for (int a = 0; a < q->num_aggregations; ++a) {
    const ph_aggregation& g = q->aggregations[a];
    k += std::to_string(g.type) + "," + std::to_string(g.log2m) + "," + std::to_string(g.expr_op) + ",";
    add(g.column);
    add(g.column2);
  }
  k += "|";
  for (ph_segment* s : all) k += std::to_string(s->id) + ",";
  return k;
}

}  // namespace

// The dense layout of a query shape over a segment set (and the per-device copies of the group-by unions when the
// devices have no table-level dictionaries): a planning pass over every segment, kept per (shape, segments,
// dictionaries) so a repeated query plans it once (r5: the layout pass, the unions and the per-query allocations were
// most of the ~10 ms of host time of a --devices 0,0 config-3 step)
struct LayoutEntry {
  ph_dense_layout layout{};
  bool have_tables = true;
  std::vector<std::vector<std::shared_ptr<GlobalDict>>> dicts;  // [device][group-by column] (!have_tables)
};

struct MultiState {
  std::mutex place_mu;          // segment placement
  std::mutex comm_mu;           // communicator creation / use (one collective sequence at a time)
  std::vector<ncclComm_t> comms;  // one per device (distinct ordinals only), created on first use
  std::mutex layout_mu;
  std::map<std::string, std::shared_ptr<LayoutEntry>> layouts;  // bounded: cleared at kLayoutCacheEntries
  ~MultiState() {
    if (!comms.empty())
      for (auto c : comms) rccl().destroy(c);
  }
};

void context_init(Context& c, int ordinal) {
  int n = 0;
  PH_HIP_CHECK(hipGetDeviceCount(&n));
  if (ordinal < 0 || ordinal >= n) fail(PH_ERR_INVALID_ARGUMENT, "device ordinal " + std::to_string(ordinal) + " out of range");
  c.device = ordinal;
  PH_HIP_CHECK(hipSetDevice(ordinal));
  c.lane_release(c.lane_acquire());  // one execution lane up front (fails here, not in a query, on a bad device)
  hipDeviceProp_t prop;
  PH_HIP_CHECK(hipGetDeviceProperties(&prop, ordinal));
  c.num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
}

void multi_init(ph_ctx* x, const int32_t* ordinals, int32_t n) {
  if (!ordinals || n < 1 || n > 64) fail(PH_ERR_INVALID_ARGUMENT, "device set");
  context_init(x->c, ordinals[0]);
  x->devs = {&x->c};
  x->ordinals = {ordinals[0]};
  for (int32_t i = 1; i < n; ++i) {
    x->more.push_back(std::make_unique<Context>());
    context_init(*x->more.back(), ordinals[i]);
    x->more.back()->device_index = i;
    x->devs.push_back(x->more.back().get());
    x->ordinals.push_back(ordinals[i]);
  }
  x->multi = std::make_shared<MultiState>();
}

// PH_TRANSPORT_RCCL: one communicator per device, created once here (ncclCommInitAll), not inside a query
void multi_set_transport(ph_ctx* x, int32_t transport) {
  if (transport != PH_TRANSPORT_PEER && transport != PH_TRANSPORT_RCCL) fail(PH_ERR_INVALID_ARGUMENT, "transport");
  std::lock_guard<std::mutex> lk(x->multi->comm_mu);
  bool distinct = true;
  for (size_t a = 0; a < x->ordinals.size(); ++a)
    for (size_t b = a + 1; b < x->ordinals.size(); ++b) distinct &= x->ordinals[a] != x->ordinals[b];
  if (transport == PH_TRANSPORT_RCCL && distinct && x->devs.size() > 1 && x->multi->comms.empty()) {
    const Rccl& api = rccl();
    std::vector<ncclComm_t> comms(x->devs.size());
    nccl_check(api.init_all(comms.data(), (int)comms.size(), x->ordinals.data()), "ncclCommInitAll");
    x->multi->comms = comms;
  }
  x->transport = transport;
}

// the device a new segment of `rows` docs goes to: the fewest docs pinned so far (its rows are reserved at once, so
// concurrent pins spread too); the caller unreserves them if the pin fails
Context* place_segment(ph_ctx* x, int64_t rows) {
  if (x->devs.size() <= 1) return &x->c;
  std::lock_guard<std::mutex> lk(x->multi->place_mu);
  Context* best = x->devs[0];
  for (Context* c : x->devs)
    if (c->pinned_rows < best->pinned_rows) best = c;
  best->pinned_rows += rows;
  return best;
}

ph_result* multi_execute(ph_ctx* x, const ph_query* q, ph_segment* const* segs, int32_t nseg) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  if (!q) fail(PH_ERR_INVALID_ARGUMENT, "null query");
  const int D = (int)x->devs.size();
  std::vector<std::vector<ph_segment*>> by(D);
  std::vector<ph_segment*> all;
  for (int32_t i = 0; i < nseg; ++i) {
    ph_segment* s = segs[i];
    if (!s) fail(PH_ERR_INVALID_ARGUMENT, "null segment");
    const int k = s->ctx->device_index;
    if (k < 0 || k >= D || x->devs[k] != s->ctx) fail(PH_ERR_INVALID_ARGUMENT, "segment not pinned through this context");
    by[k].push_back(s);
    all.push_back(s);
  }
  if (q->min_segment_group_trim_size > 0 && q->num_group_by > 0 && q->num_order_by > 0)
    return segment_trim_execute(&x->c, q, segs, nseg);  // per segment, each on its own device
  std::vector<int> active;
  for (int k = 0; k < D; ++k)
    if (!by[k].empty()) active.push_back(k);
  // segments a star-tree serves are answered from their views (startree.cpp), per device, merged by value
  if (active.size() <= 1) {
    const int k = active.empty() ? 0 : active[0];
    return query_execute_impl(x->devs[k], q, by[k].data(), (int32_t)by[k].size(), nullptr);
  }
  // the layout (and the group-by unions), planned once per query shape and segment set
  const std::string lkey = layout_key(x, q, all);
  std::shared_ptr<LayoutEntry> lay;
  {
    std::lock_guard<std::mutex> lk(x->multi->layout_mu);
    auto it = x->multi->layouts.find(lkey);
    if (it != x->multi->layouts.end()) lay = it->second;
  }
  const bool fresh = !lay;
  if (fresh) {
    lay = std::make_shared<LayoutEntry>();
    // group-by dictionaries: the table-level ones where every device has them, else one union over every device's
    // segments -- a separate copy per device (their device-side caches live on that device)
    for (int g = 0; g < q->num_group_by; ++g)
      for (Context* c : x->devs) {
        std::lock_guard<std::mutex> lk(c->mu);
        lay->have_tables &= c->table_dicts.count(q->group_by[g]) > 0;
      }
    lay->dicts.resize(D);
    if (!lay->have_tables)
      for (int g = 0; g < q->num_group_by; ++g) {
        auto u = union_dictionary(q->group_by[g], all);
        for (int k = 0; k < D; ++k) {
          auto c = std::make_shared<GlobalDict>();
          c->dict = u->dict;
          c->id = next_object_id();
          lay->dicts[k].push_back(std::move(c));
        }
      }
  }
  const bool have_tables = lay->have_tables;
  std::vector<std::vector<std::shared_ptr<GlobalDict>>>& dicts = lay->dicts;
  auto dense = [&](int k, int op) {
    DenseArgs a{op, nullptr, 0, 0, nullptr};
    if (!have_tables) a.dicts = &dicts[k];
    return a;
  };
  // a shape the dense tables do not serve: every device runs the query on its segments, the results merge on the
  // host by group value
  auto host_merge = [&]() {
    std::vector<std::unique_ptr<ph_result>> parts(D);
    per_device(active, [&](int k) {
      PH_HIP_CHECK(hipSetDevice(x->ordinals[k]));
      parts[k].reset(query_execute_impl(x->devs[k], q, by[k].data(), (int32_t)by[k].size(), nullptr));
    });
    std::vector<std::unique_ptr<ph_result>> live;
    for (auto& p : parts)
      if (p) live.push_back(std::move(p));
    ph_result* r = merge_results_by_value(q, live);
    r->stats.num_devices = (int32_t)active.size();
    r->stats.host_ms = ms_since(t0);
    return r;
  };
  if (star_tree_serves_any(q, all.data(), (int32_t)all.size())) return host_merge();
  if (fresh) {
    try {
      DenseArgs la = dense(active[0], DENSE_LAYOUT);
      la.layout = &lay->layout;
      query_execute_impl(x->devs[active[0]], q, by[active[0]].data(), (int32_t)by[active[0]].size(), &la);
    } catch (const Error& e) {
      if (e.code != PH_ERR_UNSUPPORTED) throw;
      lay->layout.num_groups = -1;  // remembered: this shape merges by value
    }
    std::lock_guard<std::mutex> lk(x->multi->layout_mu);
    if (x->multi->layouts.size() >= kLayoutCacheEntries) x->multi->layouts.clear();
    x->multi->layouts[lkey] = lay;
  }
  const ph_dense_layout& L = lay->layout;
  if (L.num_groups < 0) return host_merge();
  if (x->c.has(OPT_MULTI_HOST_MERGE)) return host_merge();  // the value-keyed merge, forced (tests)
  const int64_t G = L.num_groups;
  if (G <= 0) return host_merge();
  // shard S of every device: a multiple of 64 groups, D shards covering the padded tables
  int64_t S = (G + D - 1) / D;
  S = (S + 63) / 64 * 64;
  const int64_t padded = S * D;
  // ---- scan: every device fills its tables (identities where it has no segment, and in the padding rows); the
  // tables come from the devices' scratch pools (no hipMalloc / hipFree per query), and the identity fill of the rows
  // the scan never writes runs beside the scan on a stream of its own, drained before the merge reads them
  std::vector<std::vector<ScratchHold>> T(D);
  std::vector<ph_exec_stats> st(D);
  std::vector<int> every(D);
  for (int k = 0; k < D; ++k) every[k] = k;
  const auto t_plan = clock::now();
  per_device(every, [&](int k) {
    Context& c = *x->devs[k];
    PH_HIP_CHECK(hipSetDevice(c.device));
    std::vector<void*> ptrs;
    for (int t = 0; t < L.num_tables; ++t) {
      T[k].emplace_back(&c, (size_t)padded * L.elems_per_group[t] * L.elem_bytes[t]);
      ptrs.push_back(T[k].back().ptr());
    }
    LaneGuard lg(&c);
    const hipStream_t sk = lg.lane->stream;
    const int64_t live = by[k].empty() ? 0 : G;
    for (int t = 0; t < L.num_tables; ++t) {
      const int64_t per = L.elems_per_group[t];
      launch_fill_identity(static_cast<uint8_t*>(ptrs[t]) + (size_t)live * per * L.elem_bytes[t], (padded - live) * per,
                           L.reduce_op[t], sk);
    }
    if (!by[k].empty()) {
      DenseArgs ea = dense(k, DENSE_EXECUTE);
      ea.tables = ptrs.data();
      std::unique_ptr<ph_result> r(query_execute_impl(&c, q, by[k].data(), (int32_t)by[k].size(), &ea));
      st[k] = r->stats;
    }
    PH_HIP_CHECK(hipStreamSynchronize(sk));
  });
  const auto t_scan = clock::now();
  // ---- merge: a reduce-scatter of every table by key shard, so device k owns the fully merged shard [k S, (k + 1) S)
  //   RCCL: ncclReduceScatter over xGMI (distinct ordinals, transport PH_TRANSPORT_RCCL);
  //   PEER (default, and the only form for logical shards sharing a device): device k gathers shard k of every other
  //   device's tables by peer copy (a device-local copy when the ordinals coincide) and folds each into its own
  //   shard with k_reduce_table -- the same result as the collective, built from copies the driver always supports
  bool distinct = true;
  for (int a = 0; a < D; ++a)
    for (int b = a + 1; b < D; ++b) distinct &= x->ordinals[a] != x->ordinals[b];
  const bool use_rccl = distinct && x->transport == PH_TRANSPORT_RCCL;
  std::vector<std::pair<int, std::pair<int64_t, int64_t>>> shards;  // (device, [g0, g1)) to finalise
  std::vector<std::vector<ScratchHold>> R(D);  // reduce-scatter outputs
  for (int k = 0; k < D; ++k) {
    PH_HIP_CHECK(hipSetDevice(x->ordinals[k]));
    for (int t = 0; t < L.num_tables; ++t) R[k].emplace_back(x->devs[k], (size_t)S * L.elems_per_group[t] * L.elem_bytes[t]);
  }
  if (use_rccl) {
    const Rccl& api = rccl();
    std::lock_guard<std::mutex> lk(x->multi->comm_mu);
    if (x->multi->comms.empty()) fail(PH_ERR_DEVICE, "RCCL transport without communicators");
    std::vector<std::unique_ptr<LaneGuard>> lanes;
    for (int k = 0; k < D; ++k) {
      PH_HIP_CHECK(hipSetDevice(x->ordinals[k]));
      lanes.push_back(std::make_unique<LaneGuard>(x->devs[k]));
    }
    // one reduce-scatter per table: device k receives the merged key shard [k S, (k + 1) S)
    nccl_check(api.group_start(), "ncclGroupStart");
    for (int t = 0; t < L.num_tables; ++t)
      for (int k = 0; k < D; ++k)
        nccl_check(api.reduce_scatter(T[k][t].ptr(), R[k][t].ptr(), (size_t)S * L.elems_per_group[t],
                                      nccl_type(L.reduce_op[t]), nccl_op(L.reduce_op[t]), x->multi->comms[k],
                                      lanes[k]->lane->stream),
                   "ncclReduceScatter");
    nccl_check(api.group_end(), "ncclGroupEnd");
    for (int k = 0; k < D; ++k) {
      PH_HIP_CHECK(hipSetDevice(x->ordinals[k]));
      PH_HIP_CHECK(hipStreamSynchronize(lanes[k]->lane->stream));
    }
  } else {
    per_device(every, [&](int k) {
      Context& c = *x->devs[k];
      PH_HIP_CHECK(hipSetDevice(c.device));
      LaneGuard lg(&c);
      const hipStream_t sk = lg.lane->stream;
      // one staging block per table (all copies and folds in flight on one stream, drained once at the end)
      std::vector<ScratchHold> tmp;
      for (int t = 0; t < L.num_tables; ++t) {
        const size_t eb = (size_t)L.elems_per_group[t] * L.elem_bytes[t];
        const size_t bytes = (size_t)S * eb;
        bool first = true;
        for (int j = 0; j < D; ++j) {
          const uint8_t* src = static_cast<const uint8_t*>(T[j][t].ptr()) + (size_t)k * S * eb;
          if (first) {  // device j's shard k seeds the output (identities where j has no segments)
            PH_HIP_CHECK(hipMemcpyPeerAsync(R[k][t].ptr(), c.device, src, x->ordinals[j], bytes, sk));
            first = false;
            continue;
          }
          if (by[j].empty()) continue;  // identities only
          tmp.emplace_back(&c, bytes);
          PH_HIP_CHECK(hipMemcpyPeerAsync(tmp.back().ptr(), c.device, src, x->ordinals[j], bytes, sk));
          launch_reduce_table(R[k][t].ptr(), tmp.back().ptr(), (int64_t)S * L.elems_per_group[t], L.reduce_op[t], sk);
        }
      }
      PH_HIP_CHECK(hipStreamSynchronize(sk));
    });
  }
  for (int k = 0; k < D; ++k) {
    const int64_t g0 = std::min<int64_t>(G, k * S), g1 = std::min<int64_t>(G, g0 + S);
    if (g1 > g0) shards.push_back({k, {g0, g1}});
  }
  const auto t_merge = clock::now();
  // ---- finalise the shards in parallel (a shard on a device without segments moves to the first active device)
  std::vector<std::unique_ptr<ph_result>> parts(shards.size());
  std::vector<int> idx(shards.size());
  for (size_t i = 0; i < shards.size(); ++i) idx[i] = (int)i;
  per_device(idx, [&](int i) {
    int k = shards[i].first;
    const int64_t g0 = shards[i].second.first, g1 = shards[i].second.second;
    std::vector<void*> ptrs;
    std::vector<ScratchHold> moved;
    for (int t = 0; t < L.num_tables; ++t) ptrs.push_back(R[k][t].ptr());
    if (by[k].empty()) {
      const int to = active[0];
      PH_HIP_CHECK(hipSetDevice(x->ordinals[to]));
      for (int t = 0; t < L.num_tables; ++t) {
        const size_t bytes = (size_t)(g1 - g0) * L.elems_per_group[t] * L.elem_bytes[t];
        moved.emplace_back(x->devs[to], bytes);
        PH_HIP_CHECK(hipMemcpyPeer(moved.back().ptr(), x->ordinals[to], ptrs[t], x->ordinals[k], bytes));
        ptrs[t] = moved.back().ptr();
      }
      // a device-to-device copy may return before it lands, and the finalize below runs on a non-blocking lane
      // stream that does not order after the null stream: wait for the copies (r6: the first rows of a moved shard
      // were intermittently read stale)
      PH_HIP_CHECK(hipStreamSynchronize(nullptr));
      k = to;
    }
    PH_HIP_CHECK(hipSetDevice(x->ordinals[k]));
    DenseArgs fa = dense(k, DENSE_FINALIZE);
    fa.tables = ptrs.data();
    fa.g0 = g0;
    fa.g1 = g1;
    parts[i].reset(query_execute_impl(x->devs[k], q, by[k].data(), (int32_t)by[k].size(), &fa));
  });
  const auto t_fin = clock::now();
  // ---- one result: the shards' groups back to back (ascending key ranges), the devices' scan statistics
  auto out = std::make_unique<ph_result>();
  ph_result& f = *parts[0];
  out->key_types = f.key_types;
  out->key_entry_size = f.key_entry_size;
  out->agg_types = f.agg_types;
  out->agg_log2m = f.agg_log2m;
  out->mode = f.mode;
  int64_t total = 0;
  for (auto& p : parts) total += p->num_groups;
  out->num_groups = total;
  out->keys.resize(f.keys.size());
  out->aggs.resize(f.aggs.size());
  // the shards' columns back to back in pinned blocks of the first context's pool (already mapped: no page faults on
  // a fresh 40 MB host allocation, no zero fill), copied by a few threads in 4 MiB pieces
  out->ctx = &x->c;
  struct Piece {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
  };
  std::vector<Piece> pieces;
  auto concat = [&](std::vector<ResultBuf> ph_result::*field, size_t i) {
    size_t bytes = 0;
    for (auto& p : parts) bytes += ((*p).*field)[i].size();
    ResultBuf& dst = (out.get()->*field)[i];
    if (bytes == 0) return;
    dst.pinned = x->c.pinned_acquire(bytes, &dst.cap);
    dst.n = bytes;
    size_t o = 0;
    for (auto& p : parts) {
      const ResultBuf& src = ((*p).*field)[i];
      for (size_t a = 0; a < src.size(); a += (size_t)4 << 20)
        pieces.push_back({dst.data() + o + a, src.data() + a, std::min<size_t>((size_t)4 << 20, src.size() - a)});
      o += src.size();
    }
  };
  for (size_t i = 0; i < f.keys.size(); ++i) concat(&ph_result::keys, i);
  for (size_t i = 0; i < f.aggs.size(); ++i) concat(&ph_result::aggs, i);
  pool_run(pieces.size(), 8, [&](size_t t) { std::memcpy(pieces[t].dst, pieces[t].src, pieces[t].n); });
  ph_exec_stats& s = out->stats;
  for (auto& p : parts) {  // matched docs from the merged COUNT table, shard by shard (as ph_dense_finalize)
    s.num_docs_scanned += p->stats.num_docs_scanned;
    s.num_entries_scanned_post_filter += p->stats.num_entries_scanned_post_filter;
  }
  for (int k : active) {
    const ph_exec_stats& a = st[k];
    s.num_entries_scanned_in_filter += a.num_entries_scanned_in_filter;
    s.num_total_docs += a.num_total_docs;
    s.num_segments_processed += a.num_segments_processed;
    s.num_segments_matched += a.num_segments_matched;
    s.num_groups_limit_reached |= a.num_groups_limit_reached;
    s.sum_precision_flag |= a.sum_precision_flag;
    s.device_ms = std::max(s.device_ms, a.device_ms);  // the devices scan concurrently
    s.plan_mode = a.plan_mode;
    s.scan_kernel = a.scan_kernel;
    s.limit_pass = std::max(s.limit_pass, a.limit_pass);
  }
  for (auto& p : parts) s.sum_precision_flag |= p->stats.sum_precision_flag;
  s.num_devices = (int32_t)active.size();
  s.scan_ms = std::chrono::duration<double, std::milli>(t_scan - t_plan).count();
  s.merge_ms = std::chrono::duration<double, std::milli>(t_merge - t_scan).count();
  s.finalize_ms = std::chrono::duration<double, std::milli>(t_fin - t_merge).count();
  s.host_ms = ms_since(t0);
  return out.release();
}

}  // namespace ph

ph_ctx::~ph_ctx() { multi.reset(); }
