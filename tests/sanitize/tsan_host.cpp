// tsan_host.cpp -- ThreadSanitizer run of the library's host concurrency (test infrastructure):
//  1. the filter statistic's host pool (host_pool.h pool_run, as query.cpp runs it) over filter_sim.cpp's iterator
//     simulation of random AND / OR / NOT trees on shared leaf bitmaps, 8 threads; every result must equal the
//     one-thread run;
//  2. multi.cpp's per-device phases (host_pool.h per_device) with a stub transport: each "device" fills its own
//     partial table, then every device reduces its key shard of all the others' tables (the peer transport's access
//     pattern: concurrent reads of the other devices' tables, writes to its own shard only), with the communicator
//     created once under a mutex by whichever device gets there first (MultiState::comm_mu), and one device's
//     exception rethrown after the join.  The merged table must equal the sequential sum.
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <random>
#include <stdexcept>
#include <vector>

#include "host_pool.h"
#include "ph_internal.h"

namespace ph {
[[noreturn]] void fail(int code, const std::string& msg) { throw Error{code, msg}; }
}  // namespace ph

using namespace ph;

static SimNode random_tree(std::mt19937_64& r, int nleaves, int depth) {
  SimNode n;
  if (depth == 0 || r() % 3 == 0) {
    n.op = SIM_LEAF;
    n.leaf = (int)(r() % (unsigned)nleaves);
    n.priority = 500;
    return n;
  }
  const int kind = (int)(r() % 3);
  n.op = kind == 0 ? SIM_AND : (kind == 1 ? SIM_OR : SIM_NOT);
  n.priority = kind == 0 ? 300 : 400;
  const int kids = n.op == SIM_NOT ? 1 : 2 + (int)(r() % 2);
  for (int i = 0; i < kids; ++i) n.kids.push_back(random_tree(r, nleaves, depth - 1));
  return n;
}

int main() {
  // ---- 1. the simulation pool
  std::mt19937_64 r(20251018);
  const int nleaves = 5;
  const int64_t ndocs = 20000, nw = (ndocs + 63) / 64;
  std::vector<std::vector<uint64_t>> bits(nleaves, std::vector<uint64_t>((size_t)nw));
  for (int l = 0; l < nleaves; ++l)
    for (auto& w : bits[l]) w = r() & r() & (l % 2 ? r() : ~0ull);
  for (auto& b : bits) b.back() &= (1ull << (ndocs % 64)) - 1ull;
  std::vector<SimLeaf> leaves(nleaves);
  for (int l = 0; l < nleaves; ++l) leaves[l] = {l % 3 == 2 ? SIM_BITMAP : SIM_SCAN, bits[l].data()};
  std::vector<SimNode> trees;
  for (int t = 0; t < 48; ++t) trees.push_back(random_tree(r, nleaves, 3));
  std::vector<int64_t> seq(trees.size()), par(trees.size());
  for (size_t t = 0; t < trees.size(); ++t) seq[t] = simulate_filter_entries(trees[t], leaves, ndocs);
  pool_run(trees.size(), 8, [&](size_t t) { par[t] = simulate_filter_entries(trees[t], leaves, ndocs); });
  for (size_t t = 0; t < trees.size(); ++t)
    if (seq[t] != par[t]) {
      printf("pool: tree %zu differs (%lld vs %lld)\n", t, (long long)par[t], (long long)seq[t]);
      return 1;
    }
  printf("pool: %zu simulations on 8 threads equal the 1-thread run\n", trees.size());

  // ---- 2. per-device phases with a stub transport
  const int D = 4;
  const int64_t G = 10007, S = ((G + D - 1) / D + 63) / 64 * 64;
  std::vector<std::vector<int64_t>> T(D, std::vector<int64_t>((size_t)(S * D), 0)), R(D);
  std::vector<int> every(D);
  for (int k = 0; k < D; ++k) every[k] = k;
  per_device(every, [&](int k) {  // scan: device k fills its own table
    std::mt19937_64 rk(100 + k);
    for (int64_t g = 0; g < G; ++g) T[k][(size_t)g] = (int64_t)(rk() % 1000);
  });
  std::mutex comm_mu;
  int comm_created = 0;
  per_device(every, [&](int k) {  // merge: device k reduces key shard k of every table into its own buffer
    {
      std::lock_guard<std::mutex> lk(comm_mu);
      if (!comm_created) comm_created = 1;  // the communicator, once
    }
    std::vector<int64_t>& out = R[k];
    out.assign((size_t)S, 0);
    for (int j = 0; j < D; ++j)
      for (int64_t g = 0; g < S; ++g) out[(size_t)g] += T[j][(size_t)(k * S + g)];
  });
  for (int64_t g = 0; g < G; ++g) {
    int64_t want = 0;
    for (int j = 0; j < D; ++j) want += T[j][(size_t)g];
    if (R[(size_t)(g / S)][(size_t)(g % S)] != want) {
      printf("per_device: group %lld differs\n", (long long)g);
      return 1;
    }
  }
  bool threw = false;
  try {
    per_device(every, [&](int k) {
      if (k == 2) throw Error{PH_ERR_DEVICE, "device 2 failed"};
    });
  } catch (const Error& e) {
    threw = e.msg == "device 2 failed";
  }
  if (!threw) {
    printf("per_device: the worker's exception was not rethrown\n");
    return 1;
  }
  printf("per_device: %d devices, sharded merge equals the sequential sum, exception rethrown after the join\n", D);
  return 0;
}
