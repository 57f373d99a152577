// hc_util.hpp — small host-side helpers shared by the C ABI translation units.
#pragma once
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
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
// sizes: the measured GPU/host crossover per call of 4 KiB blocks on one
// MI355X box, one caller and four concurrent ones, pageable and pinned
// (tools/crossover.py, profiles/r4/r4b/).  A GPU batch costs
// 35-110 us before its first byte moves (pipeline lease, H2D, launch, D2H,
// the framing or copy-out tasks); the host path hashes 16 GiB/s per caller.
// Each is overridable per call by its HC_*_GPU_MIN_BLOCKS.
constexpr uint64_t kAddCrcsGpuMinBlocks = 2048;  // hc_add_crcs (output blocks; 1024: host 280 / GPU 309 us)
constexpr uint64_t kReadGpuMinBlocks = 1024;     // hc_read_from_disk[_v] (blocks to hash; 1024: 281 / 220 us)
constexpr uint64_t kWalGpuMinBlocks = 1024;      // hc_wal_replay[_v] (blocks to verify; 1024: 354 / 338 us)

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

// A process-wide pool of worker threads behind parallel_for.  Spawning and
// joining threads per call cost 200-400 us per host batch on the GPU box
// (tools/crossover.py, profiles/r4/r4a/: a 16-block AddCRCsToData took 450 us
// on its GPU path, 30 us for the batched verify that spawns none), which set
// the GPU/host crossover of the host entries at thousands of blocks.
//
// A job is n tasks fn(0..n-1).  The caller posts it and takes tasks itself;
// idle workers take the others.  The caller then unposts the job and waits
// until every worker that took it has finished: it only ever waits for tasks
// that are running, so a parallel_for inside a task (a worker posting its own
// job) cannot deadlock, even with every worker busy -- the poster then runs
// all of its tasks itself.  Tasks must not wait for each other.  Workers are
// started lazily (up to kMaxWorkers) and live for the process (the pool is
// never destroyed: no thread joins during static destruction).
class TaskPool {
 public:
  static TaskPool &get() {
    static TaskPool *p = new TaskPool;
    return *p;
  }
  template <class F>
  void run(int n, F &fn) {
    Job j;
    j.n = n;
    j.call = [](void *f, int t) { (*static_cast<F *>(f))(t); };
    j.fn = &fn;
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(&j);
      const int want = std::min(kMaxWorkers, (int)workers_ + n - 1 - idle_);
      while ((int)workers_ < want) {
        std::thread([this] { work(); }).detach();
        workers_++;
        idle_++;  // (counted idle until it waits: avoids over-spawning)
      }
    }
    cv_.notify_all();
    for (int t; (t = j.next.fetch_add(1, std::memory_order_relaxed)) < n;) j.call(j.fn, t);
    std::unique_lock<std::mutex> lk(mu_);
    for (size_t k = 0; k < q_.size(); k++)
      if (q_[k] == &j) {
        q_.erase(q_.begin() + (long)k);
        break;
      }
    done_.wait(lk, [&] { return j.refs == 0; });
  }

 private:
  static constexpr int kMaxWorkers = 64;
  struct Job {
    void (*call)(void *, int) = nullptr;
    void *fn = nullptr;
    int n = 0;
    int refs = 0;  // workers inside the job (under mu_)
    std::atomic<int> next{0};
  };
  void work() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return !q_.empty(); });
      Job *j = q_.front();
      j->refs++;
      idle_--;
      lk.unlock();
      for (int t; (t = j->next.fetch_add(1, std::memory_order_relaxed)) < j->n;) j->call(j->fn, t);
      lk.lock();
      idle_++;
      if (!q_.empty() && q_.front() == j) q_.pop_front();  // all of it taken: unpost
      if (--j->refs == 0) done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::deque<Job *> q_;
  int workers_ = 0, idle_ = 0;
};

// fn(t) for t = 0 .. threads-1 on the pool (the caller takes tasks too)
template <class F>
void parallel_for(int threads, F &&fn) {
  if (threads <= 1) {
    fn(0);
    return;
  }
  TaskPool::get().run(threads, fn);
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
