// ks_parallel.h — host worker threads for the snapshot decode / encode (ks_json.h, ks_host.cpp).
// A call splits [0, n) into chunks that threads claim in order; the first exception any chunk throws is
// rethrown in the caller after every thread has joined.  Threads: KS_HOST_THREADS, else the hardware's,
// capped at 16 (one GPU's share of a node's cores).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

namespace ks {

inline int parallel_threads() {
  static const int n = [] {
    if (const char* e = std::getenv("KS_HOST_THREADS")) return std::max(1, std::atoi(e));
    const int hw = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(hw > 0 ? hw : 1, 16));
  }();
  return n;
}

template <class F>
void parallel_for(int n, int grain, F&& f) {
  const int T = std::min(parallel_threads(), std::max(1, n / std::max(grain, 1)));
  if (T <= 1) {
    for (int i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<int> next{0};
  std::exception_ptr err;
  std::mutex mu;
  const int chunk = std::max(1, std::min(grain, n / (T * 4) + 1));
  auto work = [&]() {
    try {
      for (;;) {
        const int b = next.fetch_add(chunk);
        if (b >= n) return;
        const int e = std::min(n, b + chunk);
        for (int i = b; i < e; i++) f(i);
      }
    } catch (...) {
      std::lock_guard<std::mutex> g(mu);
      if (!err) err = std::current_exception();
      next.store(n);
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < T; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  if (err) std::rethrow_exception(err);
}

}  // namespace ks
