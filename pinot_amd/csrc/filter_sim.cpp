// filter_sim.cpp -- numEntriesScannedInFilter of one segment by running the reference's doc-id iterator tree over
// per-leaf doc bitmaps (64 docs per word, doc d at bit d & 63 of word d >> 6).
//
// The statistic is the number of docs every SVScanDocIdIterator examines (SVScanDocIdIterator.java:76-142), which
// depends on how the tree drives it: next() in 256-doc batches, advance(t) doc by doc from t, applyAnd over exactly the
// docs it is given.  The tree is built the way the reference builds it from the planned filter operators:
//   BaseFilterOperator.getTrues / getFalses -- NOT swaps them (NotFilterOperator.java:52-63), AND.getFalses is an
//   OrDocIdSet of the children's falses and OR.getFalses an AndDocIdSet of them (AndFilterOperator.java:58-69,
//   OrFilterOperator.java:59-69), a leaf's falses a NotDocIdSet (BaseFilterOperator.java:104-111);
//   AndDocIdSet.iterator (:71-185): sorted / bitmap-based children merged, the scans applied to them one after another
//   (applyAnd), the rest leap-frogged by AndDocIdIterator (:38-75) behind a RangelessBitmapDocIdIterator;
//   OrDocIdSet.iterator (:61-126): two or more index-based children merged into a BitmapDocIdIterator, OrDocIdIterator
//   (:41-126) over it and the rest;  NotDocIdIterator (:29-70), whose constructor already calls its child's next();
//   AND children in FilterOperatorUtils.reorderAndFilterChildOperators order (stable, by priority: :197-241).
// DocIdSetOperator (:59-86) drains the root iterator with next() until EOF.
//
// Cost: proportional to the iterator calls the reference makes (each next-match search is a word scan), so it is the
// general path for the statistic; the common shapes have closed forms or device passes (query.cpp).
#include <algorithm>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "ph_internal.h"

namespace ph {

namespace {

constexpr int64_t kEof = INT32_MIN;  // Constants.EOF

struct Bits {  // a doc bitmap (owned or borrowed)
  const uint64_t* w = nullptr;
  std::shared_ptr<std::vector<uint64_t>> own;
  int64_t nw = 0, n = 0;
  // first doc >= x, or -1
  int64_t next(int64_t x) const {
    if (x >= n) return -1;
    int64_t i = x >> 6;
    uint64_t v = w[i] & (~0ull << (x & 63));
    while (!v) {
      if (++i >= nw) return -1;
      v = w[i];
    }
    const int64_t d = i * 64 + __builtin_ctzll(v);
    return d < n ? d : -1;
  }
};

Bits owned(std::vector<uint64_t> v, int64_t n) {
  Bits b;
  b.own = std::make_shared<std::vector<uint64_t>>(std::move(v));
  b.w = b.own->data();
  b.nw = (int64_t)b.own->size();
  b.n = n;
  return b;
}

enum ItKind { IK_SCAN, IK_SORTED, IK_BITMAP, IK_AND, IK_OR, IK_NOT };

struct It {
  ItKind kind;
  explicit It(ItKind k) : kind(k) {}
  virtual ~It() = default;
  virtual int64_t next() = 0;
  virtual int64_t advance(int64_t t) = 0;
  virtual void drain() = 0;  // next() until EOF
};
using ItPtr = std::unique_ptr<It>;

struct ScanIt : It {  // SVScanDocIdIterator
  Bits m;
  int64_t next_doc = 0, bpos = 0, bend = 0;  // the current batch's unreturned docs are matches in [bpos, bend)
  bool batch = false;
  int64_t* entries;
  ScanIt(Bits b, int64_t* e) : It(IK_SCAN), m(std::move(b)), entries(e) {}
  int64_t next() override {
    if (batch) {
      const int64_t d = m.next(bpos);
      if (d >= 0 && d < bend) {
        bpos = d + 1;
        return d;
      }
      batch = false;
    }
    // 256-doc batches from next_doc until one holds a match; every batch is counted whole
    const int64_t d = m.next(next_doc);
    if (d < 0) {
      *entries += std::max<int64_t>(0, m.n - next_doc);
      next_doc = std::max(next_doc, m.n);
      return kEof;
    }
    const int64_t start = next_doc + ((d - next_doc) / 256) * 256, end = std::min(start + 256, m.n);
    *entries += end - next_doc;
    next_doc = end;
    batch = true;
    bpos = d + 1;
    bend = end;
    return d;
  }
  int64_t advance(int64_t t) override {
    next_doc = t;
    batch = false;  // _firstMismatch = 0
    if (t >= m.n) return kEof;
    const int64_t d = m.next(t);
    if (d >= 0) {
      *entries += d - t + 1;
      next_doc = d + 1;
      return d;
    }
    *entries += m.n - t;
    next_doc = m.n;
    return kEof;
  }
  void drain() override {
    *entries += std::max<int64_t>(0, m.n - next_doc);
    next_doc = std::max(next_doc, m.n);
    batch = false;
  }
  Bits apply_and(const Bits& docs) {  // ScanBasedDocIdIterator.applyAnd
    std::vector<uint64_t> out((size_t)docs.nw);
    int64_t c = 0;
    for (int64_t i = 0; i < docs.nw; ++i) {
      c += __builtin_popcountll(docs.w[i]);
      out[(size_t)i] = docs.w[i] & m.w[i];
    }
    *entries += c;
    return owned(std::move(out), docs.n);
  }
};

struct IdxIt : It {  // SortedDocIdIterator / BitmapDocIdIterator / RangelessBitmapDocIdIterator
  Bits docs;
  int64_t cur = 0;
  IdxIt(Bits b, ItKind k) : It(k), docs(std::move(b)) {}
  int64_t next() override {
    const int64_t d = docs.next(cur);
    if (d < 0) {
      cur = docs.n;
      return kEof;
    }
    cur = d + 1;
    return d;
  }
  int64_t advance(int64_t t) override {
    cur = std::max(cur, t);
    return next();
  }
  void drain() override { cur = docs.n; }
};

struct AndIt : It {  // AndDocIdIterator
  std::vector<ItPtr> its;
  int64_t next_doc = 0;
  explicit AndIt(std::vector<ItPtr> v) : It(IK_AND), its(std::move(v)) {}
  int64_t next() override {
    int64_t max_doc = next_doc;
    int max_idx = -1, i = 0;
    const int k = (int)its.size();
    while (i < k) {
      if (i == max_idx) {
        ++i;
        continue;
      }
      const int64_t d = its[(size_t)i]->advance(max_doc);
      if (d == kEof) return kEof;
      if (d == max_doc) {
        ++i;
      } else {
        max_doc = d;
        max_idx = i;
        i = 0;
      }
    }
    next_doc = max_doc + 1;
    return max_doc;
  }
  int64_t advance(int64_t t) override {
    next_doc = t;
    return next();
  }
  void drain() override {
    while (next() != kEof) {
    }
  }
};

struct OrIt : It {  // OrDocIdIterator
  std::vector<ItPtr> its;
  std::vector<int64_t> cur;
  size_t live;
  int64_t prev = -1;
  explicit OrIt(std::vector<ItPtr> v) : It(IK_OR), its(std::move(v)), cur(its.size(), -1), live(its.size()) {}
  int64_t step(bool adv, int64_t t) {
    int64_t best = INT64_MAX;
    bool ex = false;
    for (size_t i = 0; i < live; ++i) {
      int64_t d = cur[i];
      if (adv ? d < t : d == prev) {
        d = adv ? its[i]->advance(t) : its[i]->next();
        cur[i] = d;
        if (d == kEof) {
          ex = true;
          continue;
        }
      }
      best = std::min(best, d);
    }
    if (ex) {  // removeExhaustedIterators: the last live iterator moves into the hole
      for (size_t i = 0; i < live;) {
        if (cur[i] == kEof) {
          --live;
          std::swap(its[i], its[live]);
          cur[i] = cur[live];
        } else {
          ++i;
        }
      }
    }
    if (best == INT64_MAX) return kEof;
    prev = best;
    return best;
  }
  int64_t next() override { return step(false, 0); }
  int64_t advance(int64_t t) override { return step(true, t); }
  void drain() override {  // every live child is driven to EOF by next()
    for (size_t i = 0; i < live; ++i) its[i]->drain();
    live = 0;
  }
};

struct NotIt : It {  // NotDocIdIterator
  ItPtr child;
  int64_t n, next_doc = 0, next_non;
  NotIt(ItPtr c, int64_t nd) : It(IK_NOT), child(std::move(c)), n(nd) {
    const int64_t d = child->next();
    next_non = d == kEof ? n : d;
  }
  int64_t next() override {
    while (next_doc == next_non) {
      ++next_doc;
      const int64_t d = child->next();
      next_non = d == kEof ? n : d;
    }
    if (next_doc >= n) return kEof;
    return next_doc++;
  }
  int64_t advance(int64_t t) override {
    next_doc = t;
    if (t > next_non) {
      const int64_t d = child->advance(t);
      next_non = d == kEof ? n : d;
    }
    return next();
  }
  void drain() override {
    child->drain();
    next_doc = n;
  }
};

bool index_kind(const It& i) { return i.kind == IK_SORTED || i.kind == IK_BITMAP; }
const Bits& docs_of(const It& i) { return static_cast<const IdxIt&>(i).docs; }

struct Builder {
  const std::vector<SimLeaf>& leaves;
  int64_t n, nw;
  int64_t entries = 0;

  using Maker = std::function<ItPtr()>;

  Bits leaf_bits(int l) const {
    Bits b;
    b.w = leaves[(size_t)l].bits;
    b.nw = nw;
    b.n = n;
    return b;
  }

  ItPtr and_set(const std::vector<Maker>& makers) {  // AndDocIdSet.iterator
    std::vector<ItPtr> its;
    for (auto& m : makers) its.push_back(m());
    std::vector<size_t> idx, scans, rest;
    for (size_t i = 0; i < its.size(); ++i) {
      if (index_kind(*its[i])) idx.push_back(i);
      else if (its[i]->kind == IK_SCAN) scans.push_back(i);
      else rest.push_back(i);
    }
    if ((!idx.empty() && !scans.empty()) || idx.size() > 1) {
      std::vector<uint64_t> d(docs_of(*its[idx[0]]).w, docs_of(*its[idx[0]]).w + nw);
      for (size_t j = 1; j < idx.size(); ++j) {
        const uint64_t* o = docs_of(*its[idx[j]]).w;
        for (int64_t i = 0; i < nw; ++i) d[(size_t)i] &= o[i];
      }
      Bits cur = owned(std::move(d), n);
      for (size_t s : scans) cur = static_cast<ScanIt&>(*its[s]).apply_and(cur);
      ItPtr merged = std::make_unique<IdxIt>(cur, IK_BITMAP);  // RangelessBitmapDocIdIterator
      if (rest.empty()) return merged;
      std::vector<ItPtr> v;
      v.push_back(std::move(merged));
      for (size_t r : rest) v.push_back(std::move(its[r]));
      return std::make_unique<AndIt>(std::move(v));
    }
    return std::make_unique<AndIt>(std::move(its));
  }

  ItPtr or_set(const std::vector<Maker>& makers) {  // OrDocIdSet.iterator
    std::vector<ItPtr> its;
    for (auto& m : makers) its.push_back(m());
    std::vector<size_t> idx, rest;
    for (size_t i = 0; i < its.size(); ++i) (index_kind(*its[i]) ? idx : rest).push_back(i);
    if (idx.size() > 1) {
      std::vector<uint64_t> d((size_t)nw, 0);
      for (size_t j : idx) {
        const uint64_t* o = docs_of(*its[j]).w;
        for (int64_t i = 0; i < nw; ++i) d[(size_t)i] |= o[i];
      }
      ItPtr merged = std::make_unique<IdxIt>(owned(std::move(d), n), IK_BITMAP);  // BitmapDocIdIterator
      if (rest.empty()) return merged;
      std::vector<ItPtr> v;
      v.push_back(std::move(merged));
      for (size_t r : rest) v.push_back(std::move(its[r]));
      return std::make_unique<OrIt>(std::move(v));
    }
    return std::make_unique<OrIt>(std::move(its));
  }

  static int priority(const SimNode& x) {
    if (x.op == SIM_NOT) return priority(x.kids[0]);
    return x.priority;
  }

  static std::vector<const SimNode*> and_order(const SimNode& x) {
    std::vector<const SimNode*> k;
    for (auto& c : x.kids) k.push_back(&c);
    std::stable_sort(k.begin(), k.end(), [](const SimNode* a, const SimNode* b) { return priority(*a) < priority(*b); });
    return k;
  }

  Maker trues(const SimNode& x) {
    if (x.op == SIM_LEAF) {
      const int l = x.leaf;
      const int kind = leaves[(size_t)l].kind;
      if (kind == SIM_SCAN) return [this, l] { return ItPtr(std::make_unique<ScanIt>(leaf_bits(l), &entries)); };
      return [this, l, kind] { return ItPtr(std::make_unique<IdxIt>(leaf_bits(l), kind == SIM_SORTED ? IK_SORTED : IK_BITMAP)); };
    }
    if (x.op == SIM_AND) {
      std::vector<Maker> m;
      for (const SimNode* c : and_order(x)) m.push_back(trues(*c));
      return [this, m] { return and_set(m); };
    }
    if (x.op == SIM_OR) {
      std::vector<Maker> m;
      for (auto& c : x.kids) m.push_back(trues(c));
      return [this, m] { return or_set(m); };
    }
    return falses(x.kids[0]);  // NOT
  }

  Maker falses(const SimNode& x) {
    if (x.op == SIM_LEAF) {
      Maker t = trues(x);
      return [this, t] { return ItPtr(std::make_unique<NotIt>(t(), n)); };
    }
    if (x.op == SIM_AND) {
      std::vector<Maker> m;
      for (const SimNode* c : and_order(x)) m.push_back(falses(*c));
      return [this, m] { return or_set(m); };
    }
    if (x.op == SIM_OR) {
      std::vector<Maker> m;
      for (auto& c : x.kids) m.push_back(falses(c));
      return [this, m] { return and_set(m); };
    }
    return trues(x.kids[0]);
  }
};

}  // namespace

int64_t simulate_filter_entries(const SimNode& root, const std::vector<SimLeaf>& leaves, int64_t num_docs) {
  if (num_docs <= 0) return 0;
  Builder b{leaves, num_docs, (num_docs + 63) / 64};
  ItPtr it = b.trues(root)();
  it->drain();
  return b.entries;
}

// words per chunk (r5 swept 2, 4 and 8: 4 best): the LDS staging of K x (CW + 1) words per thread sets the waves per CU
// of k_and_dfa, the per-chunk walks of the other entry types (~4 epochs per chunk) the overhead of small chunks
int and_dfa_chunk_words() { return kDfaChunkWords; }

// The AND-of-scans entries by the device's algorithm (and_walk.h) on the host: chunks of 1 << shift docs (any
// length: dfa_chunk takes arbitrary bounds), their tables composed in order.
int64_t and_walk_entries_host(const uint64_t* bits, int k, int64_t num_docs, int shift) {
  if (num_docs <= 0) return 0;
  if (k < 1 || k > kMaxFbProgs) return -1;
  const int64_t nwords = (num_docs + 63) / 64;
  const int64_t L = shift >= 62 ? num_docs : std::min<int64_t>(num_docs, (int64_t)1 << shift);
  constexpr int K = kMaxFbProgs;
  unsigned long long total = 0;  // along entry type -1 only (the composed row a segment needs), in 64 bits
  int e = 0;
  for (int64_t c0 = 0; c0 < num_docs; c0 += L) {
    const int64_t c1 = std::min(num_docs, c0 + L);
    uint32_t d[K + 1];
    uint8_t x[K + 1];
    auto get = [&](int i, int64_t w) -> unsigned long long { return bits[(int64_t)i * nwords + w]; };
    dfa_chunk<K>(k, c0, c1, get, d, x);
    total += (unsigned long long)(int64_t)(int32_t)d[e];
    e = x[e];
  }
  return num_docs - 1 + (int64_t)total + (e == 0 ? 1 : 0);
}

// The same entries through k_and_dfa_reg's word tables (dfa_word, scans past k filled with all-ones words up to K)
template <int K>
static int64_t and_walk_entries_words(const uint64_t* bits, int k, int64_t num_docs) {
  const int64_t nwords = (num_docs + 63) / 64;
  unsigned long long total = 0;
  int e = 0;
  for (int64_t w = 0; w < nwords; ++w) {
    const int32_t c1 = (int32_t)std::min<int64_t>(64, num_docs - w * 64);
    unsigned long long W[K];
    for (int i = 0; i < K; ++i)
      W[i] = i < k ? bits[(int64_t)i * nwords + w] & (c1 < 64 ? (1ull << c1) - 1ull : ~0ull) : ~0ull;
    uint32_t d[K + 1];
    uint8_t x[K + 1];
    dfa_word<K>(k, W, c1, d, x);
    total += (unsigned long long)(int64_t)(int32_t)d[e];  // a word's sum is < 0 only for k = 1
    e = x[e];
  }
  return num_docs - 1 + (int64_t)total + (e == 0 ? 1 : 0);
}

}  // namespace ph

// test hook: the AND-of-scans entries by k_and_dfa_reg's per-word tables on the host, with `width` (k..4) scans
extern "C" int64_t phx_and_walk_entries_words(const uint64_t* bits, int32_t k, int64_t num_docs, int32_t width) {
  using namespace ph;
  if (num_docs <= 0) return 0;
  if (k < 1 || k > width || width > 4) return -1;
  switch (width) {
    case 1:
    case 2: return and_walk_entries_words<2>(bits, k, num_docs);
    case 3: return and_walk_entries_words<3>(bits, k, num_docs);
    default: return and_walk_entries_words<4>(bits, k, num_docs);
  }
}

// test hooks (not part of the product boundary, include/pinot_hip.h).  k_and_dfa's chunk tables composed on the host
// over k leaf bitmaps (leaf-major), so the CPU tests check the automaton against the simulator
extern "C" int64_t phx_and_walk_entries(const uint64_t* bits, int32_t k, int64_t num_docs, int32_t shift) {
  return ph::and_walk_entries_host(bits, k, num_docs, shift);
}

// test hook: the workgroup tables k_and_dfa writes (chunks of and_dfa_chunk_words() words composed per `block` chunks), on
// the host: gtab = (k + 1) x groups deltas, then (k + 1) x groups exit types + 1; returns the group count
extern "C" int64_t phx_and_walk_tables_host(const uint64_t* bits, int32_t k, int64_t num_docs, int32_t block,
                                            uint32_t* gtab) {
  using namespace ph;
  constexpr int K = kMaxFbProgs;
  const int CW = and_dfa_chunk_words();
  if (num_docs <= 0 || k < 1 || k > K || block < 1) return -1;
  const int64_t nwords = (num_docs + 63) / 64, nchunks = (num_docs + CW * 64 - 1) / (CW * 64);
  const int64_t ngroups = (nchunks + block - 1) / block;
  auto get = [&](int i, int64_t w) -> unsigned long long { return bits[(int64_t)i * nwords + w]; };
  for (int64_t g = 0; g < ngroups; ++g) {
    uint32_t d[K + 1];
    uint8_t x[K + 1];
    for (int e = 0; e <= K; ++e) {
      d[e] = 0;
      x[e] = (uint8_t)e;
    }
    for (int64_t c = g * block; c < std::min(nchunks, (g + 1) * block); ++c) {
      const int64_t c0 = c * CW * 64, c1 = std::min(num_docs, c0 + CW * 64);
      uint32_t cd[K + 1], od[K + 1];
      uint8_t cx[K + 1], ox[K + 1];
      for (int e = 0; e <= K; ++e) {
        cd[e] = 0;
        cx[e] = (uint8_t)e;
      }
      dfa_chunk<K>(k, c0, c1, get, cd, cx);
      dfa_compose<K>(k, d, x, cd, cx, od, ox);
      for (int e = 0; e <= k; ++e) {
        d[e] = od[e];
        x[e] = ox[e];
      }
    }
    for (int e = 0; e <= k; ++e) {
      gtab[(size_t)e * ngroups + g] = d[e];
      gtab[(size_t)(k + 1) * ngroups + (size_t)e * ngroups + g] = x[e];
    }
  }
  return ngroups;
}

// test hook: the simulator over a flat tree -- node i =
// (op, priority, leaf, first child, child count) -- so the CPU tests can check it against the oracle's restatement
extern "C" int64_t phx_filter_entries_sim(const int32_t* nodes, int32_t num_nodes, const int32_t* leaf_kinds,
                                          const uint64_t* const* leaf_bits, int32_t num_leaves, int64_t num_docs) {
  using namespace ph;
  std::vector<SimLeaf> leaves((size_t)num_leaves);
  for (int i = 0; i < num_leaves; ++i) leaves[(size_t)i] = {leaf_kinds[i], leaf_bits[i]};
  std::function<SimNode(int)> build = [&](int i) {
    SimNode x;
    x.op = nodes[5 * i];
    x.priority = nodes[5 * i + 1];
    x.leaf = nodes[5 * i + 2];
    for (int c = 0; c < nodes[5 * i + 4]; ++c) x.kids.push_back(build(nodes[5 * i + 3] + c));
    return x;
  };
  if (num_nodes <= 0) return 0;
  try {
    return simulate_filter_entries(build(0), leaves, num_docs);
  } catch (...) {
    return -1;
  }
}
