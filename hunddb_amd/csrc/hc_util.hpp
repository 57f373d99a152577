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
#include <cstdio>
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
constexpr uint64_t kAddCrcsGpuMinBlocks = 2048;  // hc_add_crcs (output blocks; 1024: host 280 / GPU 309 us)
constexpr uint64_t kReadGpuMinBlocks = 1024;     // hc_read_from_disk[_v] (blocks to hash; 1024: 281 / 220 us)
constexpr uint64_t kWalGpuMinBlocks = 1024;      // hc_wal_replay[_v] (blocks to verify; 1024: 354 / 338 us)

// The library's per-call settings ("knobs"), read from the environment ONCE,
// at the first call that needs one, and changed afterwards only through
// hc_debug_set (tests, tools/crossover.py).  Round 4 read them with getenv on
// every call; in the Go embedding os.Setenv calls setenv(3) through cgo, and a
// getenv racing with it is a glibc data race.
enum Knob : int {
  kKnobDevice,         // HC_DEVICE: the device of single-device entries (0)
  kKnobSegMinMsgs,     // HC_SEG_MIN_MSGS: whole-message device batches from this size go to k_seg_* (1)
  kKnobCopyThreads,    // HC_COPY_THREADS: host framing / copy-out tasks (8)
  kKnobWalMinRange,    // HC_WAL_MIN_RANGE: blocks per WAL scan range (64)
  kKnobAddCrcsGpuMin,  // HC_ADD_CRCS_GPU_MIN_BLOCKS (kAddCrcsGpuMinBlocks)
  kKnobReadGpuMin,     // HC_READ_GPU_MIN_BLOCKS (kReadGpuMinBlocks)
  kKnobWalGpuMin,      // HC_WAL_GPU_MIN_BLOCKS (kWalGpuMinBlocks)
  kKnobForceGpu,       // HC_FORCE_GPU: test mode, the drop-ins through the GPU and no host finish (0)
  kKnobInject,         // HC_INJECT_FAIL=<site>[:nomem]: test mode, a named GPU batch fails (0 = none)
  kKnobSegGrpMin,      // HC_SEG_GRP_MIN: records from which a refused batch may take k_crc_grp (2^18)
  kKnobSegMinBlocks,   // HC_SEG_MIN_BLOCKS: uniform device block batches k_crc_grp refuses go to k_seg_* (4096)
  kKnobSegSortMin,     // HC_SEG_SORT_MIN: records from which an unsorted batch is sorted for the stream (2^18; 0 never)
  kKnobSegSyncSpins,   // HC_SEG_SYNC_SPINS: test hook, the sort's residency-check bound in polls (2^17)
  kKnobSegSortUc,      // HC_SEG_SORT_UC: test hook, units per coarse bucket of the sort at most (0: 32768)
  kKnobSegLgChunk,     // HC_SEG_LG_CHUNK: tuning, log2 of the stream's units per chunk slot (3: 128 KiB; 0-12)
  kKnobCount
};
struct KnobDef {
  const char *env;
  int64_t dflt;
};
inline constexpr KnobDef kKnobDefs[kKnobCount] = {
    {"HC_DEVICE", 0},          {"HC_SEG_MIN_MSGS", 1},
    {"HC_COPY_THREADS", 8},    {"HC_WAL_MIN_RANGE", 64},
    {"HC_ADD_CRCS_GPU_MIN_BLOCKS", (int64_t)kAddCrcsGpuMinBlocks},
    {"HC_READ_GPU_MIN_BLOCKS", (int64_t)kReadGpuMinBlocks},
    {"HC_WAL_GPU_MIN_BLOCKS", (int64_t)kWalGpuMinBlocks},
    {"HC_FORCE_GPU", 0},       {"HC_INJECT_FAIL", 0},
    {"HC_SEG_GRP_MIN", 1 << 18}, {"HC_SEG_MIN_BLOCKS", 4096},
    {"HC_SEG_SORT_MIN", 1 << 18}, {"HC_SEG_SYNC_SPINS", 1 << 17}, {"HC_SEG_SORT_UC", 0},
    {"HC_SEG_LG_CHUNK", 3},
};
// HC_INJECT_FAIL sites, as knob values (site | 16 for :nomem)
enum : int64_t { kInjectAddCrcs = 1, kInjectReadFromDisk = 2, kInjectWalReplay = 3, kInjectNomem = 16 };
inline int64_t parse_inject(const char *v) {
  if (!v || !*v) return 0;
  static const char *const sites[] = {"add_crcs", "read_from_disk", "wal_replay"};
  for (int k = 0; k < 3; k++) {
    const size_t n = std::strlen(sites[k]);
    if (std::strncmp(v, sites[k], n) != 0) continue;
    if (v[n] == 0) return k + 1;
    if (v[n] != ':') continue;
    if (std::strcmp(v + n + 1, "nomem") == 0) return (k + 1) | kInjectNomem;
    // any other suffix keeps the site's HC_E_HIP failure (round 4's meaning of
    // "<site>:<anything>"), so a script with a typo still runs the host recovery
    std::fprintf(stderr, "hundcrc: HC_INJECT_FAIL=%s: unknown suffix, injecting HC_E_HIP at %s\n", v, sites[k]);
    return k + 1;
  }
  return 0;  // an unknown site injects nothing
}
// parse a knob's text value (the environment or hc_debug_set); nullptr/"" -> the default
inline int64_t parse_knob(int k, const char *v) {
  if (!v || !*v) return kKnobDefs[k].dflt;
  if (k == kKnobInject) return parse_inject(v);
  return std::strtoll(v, nullptr, 10);
}
inline std::atomic<int64_t> g_knobs[kKnobCount];
inline std::once_flag g_knobs_once;
inline int64_t knob(Knob k) {
  std::call_once(g_knobs_once, [] {
    for (int i = 0; i < kKnobCount; i++) g_knobs[i].store(parse_knob(i, std::getenv(kKnobDefs[i].env)));
  });
  return g_knobs[k].load(std::memory_order_relaxed);
}
// hc_debug_set: by environment name; value nullptr restores the compiled default
inline bool knob_set(const char *name, const char *value) {
  knob(kKnobDevice);  // (the environment is read first, so a set is never overwritten by it)
  for (int i = 0; i < kKnobCount; i++)
    if (name && std::strcmp(name, kKnobDefs[i].env) == 0) {
      g_knobs[i].store(parse_knob(i, value));
      return true;
    }
  return false;
}

// Process-wide event counters behind hc_stats() (defined in hc_api.cpp).
struct Stats {
  std::atomic<uint64_t> add_crcs_gpu{0}, add_crcs_host_small{0}, add_crcs_host_nodev{0}, add_crcs_gpu_fallback{0};
  std::atomic<uint64_t> read_gpu{0}, read_gpu_fallback{0}, wal_gpu{0}, wal_gpu_fallback{0}, nodev_host{0};
  std::atomic<int64_t> last_fallback_error{0};
};
extern Stats g_stats;

// The HC_INJECT_FAIL test hook: the named GPU batch reports HC_E_HIP (or
// HC_E_NOMEM) without running, so the host recovery path can be tested on any
// machine.  Returns 0 when `site` is not the one set.
inline int injected_failure(int64_t site) {
  const int64_t v = knob(kKnobInject);
  if ((v & 15) != site) return 0;
  return (v & kInjectNomem) ? -4 /*HC_E_NOMEM*/ : -2 /*HC_E_HIP*/;
}

// A GPU batch failure the host entries (AddCRCsToData, ReadFromDisk, WAL
// replay) finish on the host path: no gfx950, a device or pinned allocation
// failure, a HIP runtime error.  Any other code (HC_E_ARG, HC_E_LAYOUT: a
// caller or library bug) is returned, never hidden behind the host path.
inline bool gpu_batch_failure(int rc) { return rc == -3 /*HC_E_NODEV*/ || rc == -4 /*HC_E_NOMEM*/ || rc == -2 /*HC_E_HIP*/; }

// HC_FORCE_GPU=1 routes the single-buffer drop-ins through the GPU batch path
// too, and returns a failed GPU batch instead of finishing it on the host.
inline int force_gpu() { return (int)knob(kKnobForceGpu); }

// A process-wide pool of worker threads behind parallel_for.  Spawning and
// joining threads per call cost 200-400 us per host batch on the GPU box
// (tools/crossover.py, profiles/r4/r4a/: a 16-block AddCRCsToData took 450 us
// on its GPU path, 30 us for the batched verify that spawns none), which set
// the GPU/host crossover of the host entries at thousands of blocks.
//
// A job is n tasks fn(0..n-1).  The caller posts it, runs task 0 itself and
// then takes further tasks; idle workers take the others.  The caller then unposts the job and waits
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
    j.next.store(1, std::memory_order_relaxed);  // task 0 is the caller's (below)
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
    j.call(j.fn, 0);  // the caller runs task 0 itself: callers put the GPU batch there (thread-local launch info)
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
