// hc_util.hpp — small host-side helpers shared by the C ABI translation units.
#pragma once
#include <cstdlib>
#include <thread>
#include <vector>

namespace hc {

inline int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// HC_FORCE_GPU=1 routes the single-buffer drop-ins through the GPU batch path
// too (read per call so tests can toggle it).
inline int force_gpu() { return env_int("HC_FORCE_GPU", 0); }

// fn(t) on `threads` threads (the caller runs t = 0)
template <class F>
void parallel_for(int threads, F &&fn) {
  if (threads <= 1) {
    fn(0);
    return;
  }
  std::vector<std::thread> ts;
  ts.reserve(threads - 1);
  for (int t = 1; t < threads; t++) ts.emplace_back([&fn, t] { fn(t); });
  fn(0);
  for (auto &t : ts) t.join();
}

}  // namespace hc
