// hc_util.hpp — small host-side helpers shared by the C ABI translation units.
#pragma once
#include <emmintrin.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace hc {

inline int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// Host entries with a host path of their own switch to the GPU batch at these
// sizes (the measured GPU/host crossover per call, DESIGN.md 5.2,
// tools/crossover.py); each is overridable per call by its HC_*_GPU_MIN_BLOCKS.
constexpr uint64_t kAddCrcsGpuMinBlocks = 256;  // hc_add_crcs (output blocks)
constexpr uint64_t kReadGpuMinBlocks = 256;     // hc_read_from_disk[_v] (blocks to hash)
constexpr uint64_t kWalGpuMinBlocks = 256;      // hc_wal_replay[_v] (blocks to verify)

// Process-wide event counters behind hc_stats() (defined in hc_api.cpp).
struct Stats {
  std::atomic<uint64_t> add_crcs_gpu{0}, add_crcs_host_small{0}, add_crcs_host_nodev{0}, add_crcs_gpu_fallback{0};
  std::atomic<uint64_t> read_gpu{0}, read_gpu_fallback{0}, wal_gpu{0}, wal_gpu_fallback{0}, nodev_host{0};
  std::atomic<int64_t> last_fallback_error{0};
};
extern Stats g_stats;

// HC_INJECT_FAIL=<site>[:nomem] (read per call, tests only): the named GPU
// batch ("add_crcs", "read_from_disk", "wal_replay") reports HC_E_HIP (or
// HC_E_NOMEM) without running, so the host recovery path can be tested on any
// machine.  Returns 0 when `site` is not named.
inline int injected_failure(const char *site) {
  const char *v = std::getenv("HC_INJECT_FAIL");
  if (!v || !*v) return 0;
  const size_t n = std::strlen(site);
  if (std::strncmp(v, site, n) != 0 || (v[n] != 0 && v[n] != ':')) return 0;
  return (v[n] == ':' && std::strcmp(v + n + 1, "nomem") == 0) ? -4 /*HC_E_NOMEM*/ : -2 /*HC_E_HIP*/;
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

// Bytes written once and not read back by the CPU (framed output, staging
// that the DMA engine reads): non-temporal 16-B stores skip the write-allocate
// read of every destination line.  Weakly ordered: the writing thread issues
// _mm_sfence() before another thread or the DMA engine reads the bytes.
inline void copy_nt(uint8_t *dst, const uint8_t *src, uint64_t n) {
  if (n < 64) {
    std::memcpy(dst, src, n);
    return;
  }
  const uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  for (; n >= 64; n -= 64, dst += 64, src += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 48), d);
  }
  std::memcpy(dst, src, n);
}

}  // namespace hc
