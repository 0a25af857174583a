// host_pool.h -- the library's two host concurrency patterns, header-only so tests/sanitize/tsan_host.cpp runs the
// very same code under ThreadSanitizer:
//  * pool_run: n work items over min(n, max_threads) threads pulling indices from one atomic counter (the filter
//    statistic's host iterator simulations, query.cpp); every item writes only its own output slot;
//  * per_device: f(k) for every device k on its own thread (multi.cpp's scan / merge / finalize phases).
// Both join every thread before returning and rethrow the first exception a worker caught.
#pragma once
#include <algorithm>
#include <atomic>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

namespace ph {

template <class F>
void pool_run(size_t n, size_t max_threads, F&& f) {
  if (n == 0) return;
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> errs;
  std::mutex err_mu;
  auto work = [&]() {
    try {
      for (size_t t; (t = next.fetch_add(1)) < n;) f(t);
    } catch (...) {
      std::lock_guard<std::mutex> lk(err_mu);
      errs.push_back(std::current_exception());
    }
  };
  const size_t nthr = std::min(n, std::max<size_t>(1, max_threads));
  std::vector<std::thread> pool;
  for (size_t k = 1; k < nthr; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  if (!errs.empty()) std::rethrow_exception(errs.front());
}

template <class F>
void per_device(const std::vector<int>& ks, F&& f) {
  std::vector<std::exception_ptr> err(ks.size());
  std::vector<std::thread> th;
  for (size_t i = 0; i < ks.size(); ++i)
    th.emplace_back([&, i] {
      try {
        f(ks[i]);
      } catch (...) {
        err[i] = std::current_exception();
      }
    });
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

}  // namespace ph
