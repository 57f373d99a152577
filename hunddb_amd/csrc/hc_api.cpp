// hc_api.cpp — C ABI of libhundcrc.so (include/hundcrc.h): the drop-in
// utils/crc surface (/root/reference/utils/crc/crc_util.go:10-122) and the
// batched GPU entries, plus the host runtime behind them (per-device constant
// tables, per-thread streams, pinned staging ring with H2D/kernel/D2H overlap).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hundcrc.h"
#include "hc_gf2.hpp"
#include "hc_kernels.hpp"
#include "hc_util.hpp"

namespace hc {
uint32_t cpu_crc32_update(uint32_t crc, const uint8_t *p, size_t n);
}

using namespace hc;

namespace {

constexpr size_t kPayloadPerBlock = HC_BLOCK_SIZE - HC_CRC_SIZE;  // 4092 (crc_util.go:43)

}  // namespace

// Process-wide event counters (hc_stats; hc_wal.cpp counts its replays too).
hc::Stats hc::g_stats;

namespace {
void count_fallback(std::atomic<uint64_t> &c, int rc) {
  if (rc == HC_E_NODEV) {
    g_stats.nodev_host.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  c.fetch_add(1, std::memory_order_relaxed);
  g_stats.last_fallback_error.store(rc, std::memory_order_relaxed);
}


// ---------------------------------------------------------------------------
// Devices
struct DeviceState {
  std::once_flag once;
  int status = HC_E_NODEV;
  int cus = 0;
  DeviceTables *dtab = nullptr;  // device copy of the constant image
  SegTables *dseg = nullptr;     // the packed-record path's tables (k_seg_*)
  uint32_t *seg_last = nullptr;  // 1 when the last packed-record stream took its batch
  // off/len batches: k_crc_grp's "a block was left to the sweep" word and the
  // per-call tag it is raised to (Batch::skip_slot)
  unsigned long long *skip_slot = nullptr;
  std::atomic<uint64_t> skip_tag{0};
  // the packed-record stream's workspace for calls on the null stream, kept
  // across calls: that stream orders every use after the previous one and is
  // never destroyed.  Calls on other streams (which may be destroyed and their
  // handles reused) or under graph capture take one from the stream-ordered
  // allocator per call.  An event ordering a kept workspace across streams
  // costs what the allocator pair does (profiles/r3/seg/).
  std::mutex seg_mu;
  uint32_t *seg_ws = nullptr;
  uint64_t seg_ws_bytes = 0;
};

constexpr int kMaxDevices = 64;
DeviceState g_dev[kMaxDevices];

const SegTables &host_seg_tables() {
  static const SegTables *t = [] {
    auto *p = new SegTables;
    build_seg_tables(*p);
    return p;
  }();
  return *t;
}

const DeviceTables &host_tables() {
  static const DeviceTables *t = [] {
    auto *p = new DeviceTables;
    build_device_tables(*p);
    return p;
  }();
  return *t;
}

struct DeviceGuard {  // keep the caller's current device untouched
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int device_count_raw() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int init_device(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return HC_E_ARG;
  DeviceState &d = g_dev[dev];
  std::call_once(d.once, [&] {
    if (dev >= device_count_raw()) return;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return;  // kernels are gfx950-only
    DeviceGuard g(dev);
    void *p = nullptr;
    if (hipMalloc(&p, sizeof(DeviceTables)) != hipSuccess) {
      d.status = HC_E_NOMEM;
      return;
    }
    if (hipMemcpy(p, &host_tables(), sizeof(DeviceTables), hipMemcpyHostToDevice) != hipSuccess) {
      d.status = HC_E_HIP;
      return;
    }
    d.dtab = static_cast<DeviceTables *>(p);
    if (hipMalloc(&p, sizeof(SegTables)) != hipSuccess) {
      d.status = HC_E_NOMEM;
      return;
    }
    if (hipMemcpy(p, &host_seg_tables(), sizeof(SegTables), hipMemcpyHostToDevice) != hipSuccess) {
      d.status = HC_E_HIP;
      return;
    }
    d.dseg = static_cast<SegTables *>(p);
    if (hipMalloc(&p, 4) != hipSuccess || hipMemset(p, 0, 4) != hipSuccess) {
      d.status = HC_E_NOMEM;
      return;
    }
    d.seg_last = static_cast<uint32_t *>(p);
    if (hipMalloc(&p, 8) != hipSuccess || hipMemset(p, 0, 8) != hipSuccess) {
      d.status = HC_E_NOMEM;
      return;
    }
    d.skip_slot = static_cast<unsigned long long *>(p);

    d.cus = prop.multiProcessorCount;
    d.status = HC_OK;
  });
  return d.status;
}

int default_device() { return (int)knob(kKnobDevice); }

}  // namespace

namespace hc {
// for the other translation units (hc_merkle.cpp): init + CU count
int dev_init(int device, int *cus) {
  const int st = init_device(device);
  if (st == HC_OK && cus) *cus = g_dev[device].cus;
  return st;
}
void set_last_launch(const hc_launch_info &info);
}  // namespace hc

namespace {

thread_local hc_launch_info t_last{"", 0, 0, 0, 0, 0, 0};
thread_local int t_seg_dev = -1;  // device of this thread's last packed-record stream (hc_debug_seg_taken)

}  // namespace

void hc::set_last_launch(const hc_launch_info &info) { t_last = info; }

namespace {

// ---------------------------------------------------------------------------
// Device batch dispatch (shared by _dev_ entries and the host pipeline)
// Whole-message off/len batches with crc_out from a device entry (at least
// HC_SEG_MIN_MSGS messages, default 1: every one) first go to the packed-record
// stream (k_seg_*, launch_seg): it takes the batch when its messages lie back
// to back (off[i+1] = off[i] + len[i]) and mostly at least 64 B long, and
// raises a device flag otherwise, on which k_crc_any runs.  The decision is
// made on the device (no host sync).  On config 5's record sizes the stream
// wins at every batch size measured, 16 records up (profiles/r4/r4x/: 1.5-2.6x
// against k_crc_grp + k_crc_any); batches of up to ~1024 short records (1 KiB)
// run faster on k_crc_any (13-27 against 24-28 us: the stream's floor is its
// four launches), which a caller gets by raising HC_SEG_MIN_MSGS.  Round 3's
// default was 131072.  On the null stream the
// workspace is kept across calls (seg_cached_ws: a per-call hipMallocAsync /
// hipFreeAsync pair cost 4-17 us a call, tools/kseg3.hip); other streams take
// one from the stream-ordered allocator per call.  The span is bounded by the allocation holding
// `base` (a batch reaching past it is not packed for the stream).
uint64_t seg_min_msgs() { return (uint64_t)std::max<int64_t>(0, knob(kKnobSegMinMsgs)); }

// The kept workspace (null stream only), grown to `need` bytes on that stream,
// so the free is ordered after every earlier use.  The lock is held from here
// until the caller has enqueued the launches that use it.  nullptr: allocate
// per call.  Only workspaces up to kSegKeepBytes are kept:
// a larger one would stay pinned in the default mempool for the life of the
// process, and its per-call allocation is small against the batch.
// Relies on the legacy null stream's ordering across host threads (hundcrc.h;
// the library is not built with -fgpu-default-stream=per-thread).
constexpr uint64_t kSegKeepBytes = 512ull << 20;  // (round 6: the sort's arrays, 48 B a record: ~8M records)
uint32_t *seg_cached_ws(DeviceState &d, hipStream_t s, uint64_t need, std::unique_lock<std::mutex> &lk) {
  if (s != nullptr || need > kSegKeepBytes) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  lk = std::unique_lock<std::mutex>(d.seg_mu);
  if (d.seg_ws && d.seg_ws_bytes >= need) return d.seg_ws;
  if (d.seg_ws) (void)hipFreeAsync(d.seg_ws, s);
  d.seg_ws = nullptr;
  d.seg_ws_bytes = 0;
  const uint64_t bytes = std::min(kSegKeepBytes, need + need / 4);  // headroom for a slightly larger next batch
  if (hipMallocAsync(reinterpret_cast<void **>(&d.seg_ws), bytes, s) != hipSuccess) {
    d.seg_ws = nullptr;
    lk.unlock();
    return nullptr;
  }
  d.seg_ws_bytes = bytes;
  return d.seg_ws;
}

// Uniform device block batches that k_crc_grp cannot take (a length that is
// not a 4 KiB multiple, e.g. config.go:241's BlockSize, or an address that is
// not 16-B aligned), from HC_SEG_MIN_BLOCKS blocks: their messages block[4:]
// lie 4 + stride - ulen bytes apart, which the stream's small-gap mode takes
// (launch_seg_blocks); k_crc_any ran them at 57-62 % (round 4).
uint64_t seg_min_blocks() { return (uint64_t)std::max<int64_t>(1, knob(kKnobSegMinBlocks)); }
// The stream against k_crc_any over 4 GiB of uniform blocks, same buffers,
// alternating routes (tools/seg_blocks_sweep.py, TB/s, k_crc_any / stream).
// Round 5 (profiles/r5/r5m/, the stream's 2 MiB chunk slots): 2044 B 3.7 / 4.1,
// 4092 5.46 / 5.43, 6000 6.15 / 6.01 -- k_crc_any kept 4-B aligned blocks of
// 2-8 KiB.  Round 6 (profiles/r6/r6z/, 128 KiB slots): 1020 B 2.45-2.60 /
// 2.86-2.94, 2044 3.47-4.11 / 4.18-4.30, 4092 5.36-5.40 / 5.52-5.54, 6000
// 6.18 / 6.18-6.19, 8188 5.80 / 6.27, 16380 5.18 / 6.39-6.41, 65532 6.37 /
// 6.48-6.49; not 4-B aligned 4092 5.08 / 5.57, 8192 5.02-5.05 / 6.21-6.24:
// every length goes to the stream.

// The span bound of a batch at `base` (the allocation holding it), as k_seg_*'s unit count; 0 if unknown.
uint64_t seg_units_for(const uint8_t *base) {
  hipDeviceptr_t pb = nullptr;
  size_t ps = 0;
  if (hipMemGetAddressRange(&pb, &ps, const_cast<uint8_t *>(base)) != hipSuccess || !ps) return 0;
  const uint64_t lo = reinterpret_cast<uintptr_t>(base) & ~uint64_t(1023);
  return seg_max_units(reinterpret_cast<uintptr_t>(pb) + ps - lo);
}

// launch_seg_blocks with a kept or per-call workspace; false: not launched (no workspace)
bool seg_blocks(DeviceState &d, const Batch &b, hipStream_t s, int grid, hipError_t &e) {
  const uint64_t mu = seg_units_for(b.base);
  if (!mu) return false;
  const uint64_t need = seg_block_workspace_bytes(b.nblocks, mu, !b.crc_out);
  std::unique_lock<std::mutex> lk;
  uint32_t *ws = seg_cached_ws(d, s, need, lk), *own = nullptr;
  if (!ws && hipMallocAsync(reinterpret_cast<void **>(&own), need, s) == hipSuccess) ws = own;
  if (!ws) return false;
  e = launch_seg_blocks(b, d.dseg, ws, mu, grid, s, d.seg_last);
  if (own && hipFreeAsync(own, s) != hipSuccess && e == hipSuccess) e = hipErrorUnknown;
  return true;
}

int dispatch(int dev, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
             uint32_t ulen, uint64_t n, uint32_t *crc_out, uint32_t *bitmap, int64_t *first_bad,
             uint32_t flags, hipStream_t s, uint64_t bytes_hint, bool seg_ok = false) {
  DeviceState &d = g_dev[dev];
  Batch b{};
  b.base = base;
  b.off = off;
  b.len = len;
  b.stride = stride;
  b.ulen = ulen;
  b.flags = flags & (kFlagStamp | kFlagMessages);
  b.nblocks = n;
  b.crc_out = crc_out;
  b.bad_bitmap = bitmap;
  b.first_bad = reinterpret_cast<unsigned long long *>(first_bad);
  b.tables = d.dtab;
  if (n == 0) return HC_OK;
  t_seg_dev = -1;  // set below when the batch goes to the stream
  const int fast_grid = d.cus;  // one 1024-thread, 144 KiB-LDS workgroup per CU
  const int gen_grid = d.cus;  // k_crc_any: same geometry as the streaming kernel
  hc_launch_info info{"k_crc_fast", 0, 0, bytes_hint, (uint32_t)fast_grid, kFastThreads,
                      kFastLdsBytes};
  hipError_t e = hipSuccess;
  if (!off && !len) {
    const bool fast = ulen >= 1024 && (ulen & 1023u) == 0 &&
                      (reinterpret_cast<uintptr_t>(base) & 15u) == 0 && (stride & 15u) == 0;
    if (fast && (ulen & 4095u) == 0) {  // 4/8/16 KiB blocks: groups of 4 rows, handed out per CU
      e = launch_grp(b, fast_grid, s);
      info.kernel = "k_crc_grp";
      info.fast_blocks = n;
    } else if (fast) {
      e = launch_fast(b, fast_grid, s);
      info.fast_blocks = n;
    } else if (seg_ok && ulen >= 4 && stride >= ulen && n >= seg_min_blocks() && n < 0x7FFFFFFFull &&
               (!(flags & kFlagMessages) || crc_out) && seg_blocks(d, b, s, fast_grid, e)) {
      info.kernel = "k_seg_plan+k_seg_stream+k_seg_combine";
      info.fast_blocks = n;
      t_seg_dev = dev;
    } else {
      e = launch_general(b, 0, gen_grid, s);
      info.kernel = "k_crc_any";
      info.general_blocks = n;
    }
  } else if (!off != !len) {
    // only one of the arrays (hundcrc.h allows either): off[i] with ulen, or
    // i * stride with len[i].  k_crc_grp's contract is both arrays or neither,
    // so the whole batch takes k_crc_any, which reads each side as given.
    e = launch_general(b, 0, gen_grid, s);
    info.kernel = "k_crc_any";
    info.general_blocks = n;
  } else {
    uint32_t *seg_ws = nullptr;           // a per-call workspace (else the kept one, under seg_lock)
    std::unique_lock<std::mutex> seg_lock;  // held while the kept workspace's launches are enqueued
    bool seg = false;
    // the stream's only output is crc_out (k_seg_combine): a batch without it
    // (verify or stamp only) takes k_crc_grp + k_crc_any
    if (seg_ok && (flags & kFlagMessages) && crc_out && n >= seg_min_msgs() && n < 0x7FFFFFFFull) {
      if (const uint64_t mu = seg_units_for(base)) {
        const uint64_t sort_min = (uint64_t)std::max<int64_t>(0, knob(kKnobSegSortMin));
        const uint64_t need = seg_workspace_bytes(n, mu, sort_min && n >= sort_min);
        uint32_t *ws = seg_cached_ws(d, s, need, seg_lock);
        if (!ws && hipMallocAsync(reinterpret_cast<void **>(&seg_ws), need, s) == hipSuccess) ws = seg_ws;
        if (ws) {
          // word 0 of ws: raised when the stream did not take the batch; then
          // k_seg_combine runs k_crc_any's work over every message itself
          e = launch_seg(b, d.dseg, ws, mu, fast_grid, s, d.seg_last, (uint64_t)knob(kKnobSegGrpMin), sort_min,
                         (uint32_t)std::min<int64_t>(std::max<int64_t>(0, knob(kKnobSegSyncSpins)), 0xFFFFFFFF),
                         (uint32_t)std::min<int64_t>(std::max<int64_t>(0, knob(kKnobSegSortUc)), 0xFFFFFFFF),
                         (uint32_t)std::min<int64_t>(std::max<int64_t>(0, knob(kKnobSegLgChunk)), 12));
          seg = true;
        }
      }
    }
    if (!seg) {
      // k_crc_grp takes the 16-B aligned blocks of 4 KiB multiples (every on-disk
      // size, utils/config/config.go:137); the k_crc_any sweep does the rest
      b.skip_slot = d.skip_slot;
      b.skip_tag = d.skip_tag.fetch_add(1, std::memory_order_relaxed) + 1;
      if (e == hipSuccess) e = launch_grp(b, fast_grid, s);
      if (e == hipSuccess) e = launch_general(b, 4095, gen_grid, s);
    }
    if (seg_ws && hipFreeAsync(seg_ws, s) != hipSuccess && e == hipSuccess) e = hipErrorUnknown;
    info.kernel = seg ? "k_seg_plan+k_seg_stream+k_seg_combine" : "k_crc_grp+k_crc_any";
    t_seg_dev = seg ? dev : -1;
    info.fast_blocks = n;  // routing is decided on the device per block
  }
  t_last = info;
  return e == hipSuccess ? HC_OK : HC_E_HIP;
}

// ---------------------------------------------------------------------------
// Host-resident batches: per-thread pipeline of kSlots slots.  Each slot owns
// pinned staging, device buffers, a non-blocking stream and an event, so the
// CPU gather of chunk k+1 overlaps the H2D copy / kernel / D2H copy of the
// chunks before it.  A caller buffer that is already pinned (hipHostMalloc /
// hipHostRegister) is DMA'd directly, without the staging copy.
constexpr int kSlots = 3;

struct Slot {
  uint8_t *pin = nullptr;    // pinned staging (blocks, packed, 16-B aligned)
  uint64_t *pin_off = nullptr;
  uint32_t *pin_len = nullptr;
  uint32_t *pin_crc = nullptr;
  uint8_t *dbuf = nullptr;
  uint64_t *doff = nullptr;
  uint32_t *dlen = nullptr;
  uint32_t *dcrc = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint64_t i0 = 0, nb = 0;  // block range of the in-flight chunk
  bool busy = false;
  // MD5 batches (row f4), allocated on first use: tail workspace and digests
  uint8_t *dtail = nullptr, *dmd5 = nullptr, *pin_md5 = nullptr;
  // span-DMA target (device only, HostPipe::span bytes), allocated on first use
  uint8_t *dspan = nullptr;
  // GPU-side verify (allocated on first use): the chunk's bad-block bitmap and
  // lowest bad index, on the device and their pinned copies
  uint32_t *dbm = nullptr, *pin_bm = nullptr;
  unsigned long long *dfb = nullptr, *pin_fb = nullptr;
};

struct HostPipe {
  int dev = -1;
  int home = -1;  // the device the pool created it for
  size_t chunk = 0;   // staging bytes per slot
  size_t maxblk = 0;  // metadata capacity per slot
  size_t span = 0;    // span-DMA bytes per slot (device memory only: no pinned staging)
  Slot slot[kSlots];
  bool ok = false;

  int init(int d) {
    if (ok && dev == d) return HC_OK;
    release();
    dev = d;
    static const size_t chunk_env = (size_t)std::max(1, env_int("HC_CHUNK_MB", 64)) << 20;  // read once
    static const size_t span_env = (size_t)std::max(1, env_int("HC_SPAN_MB", 256)) << 20;
    chunk = chunk_env;
    maxblk = chunk / 64 + 1;
    // span DMA needs no pinned staging, so its chunks can be larger: fewer,
    // fuller kernels (the MD5 of one 64 MiB chunk of records is a few dozen
    // waves -- too little parallelism to keep up with the copy)
    span = std::max(chunk, span_env);
    DeviceGuard g(dev);
    for (auto &s : slot) {
      if (hipHostMalloc(reinterpret_cast<void **>(&s.pin), chunk, hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&s.pin_off), maxblk * 8, hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&s.pin_len), maxblk * 4, hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&s.pin_crc), maxblk * 4, hipHostMallocDefault) != hipSuccess ||
          hipMalloc(reinterpret_cast<void **>(&s.dbuf), chunk) != hipSuccess ||
          hipMalloc(reinterpret_cast<void **>(&s.doff), maxblk * 8) != hipSuccess ||
          hipMalloc(reinterpret_cast<void **>(&s.dlen), maxblk * 4) != hipSuccess ||
          hipMalloc(reinterpret_cast<void **>(&s.dcrc), maxblk * 4) != hipSuccess ||
          hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
        release();
        return HC_E_NOMEM;
      }
    }
    ok = true;
    return HC_OK;
  }
  void release() {
    if (dev < 0) return;
    DeviceGuard g(dev);
    for (auto &s : slot) {
      if (s.stream) (void)hipStreamSynchronize(s.stream);
      if (s.pin) (void)hipHostFree(s.pin);
      if (s.pin_off) (void)hipHostFree(s.pin_off);
      if (s.pin_len) (void)hipHostFree(s.pin_len);
      if (s.pin_crc) (void)hipHostFree(s.pin_crc);
      if (s.dbuf) (void)hipFree(s.dbuf);
      if (s.dspan) (void)hipFree(s.dspan);
      if (s.doff) (void)hipFree(s.doff);
      if (s.dlen) (void)hipFree(s.dlen);
      if (s.dcrc) (void)hipFree(s.dcrc);
      if (s.dtail) (void)hipFree(s.dtail);
      if (s.dmd5) (void)hipFree(s.dmd5);
      if (s.pin_md5) (void)hipHostFree(s.pin_md5);
      if (s.dbm) (void)hipFree(s.dbm);
      if (s.dfb) (void)hipFree(s.dfb);
      if (s.pin_bm) (void)hipHostFree(s.pin_bm);
      if (s.pin_fb) (void)hipHostFree(s.pin_fb);
      if (s.stream) (void)hipStreamDestroy(s.stream);
      if (s.done) (void)hipEventDestroy(s.done);
      s = Slot{};
    }
    ok = false;
  }
  ~HostPipe() { release(); }
};

// Process-wide pool of pipelines, at most HC_MAX_PIPES (default 4) per device: a
// host batch leases one for the duration of the call and returns it.  cgo runs
// calls on arbitrary, long-lived OS threads, so per-thread pipelines (each
// ~240 MiB pinned + ~1 GiB of device buffers) would grow with the thread
// count; here extra concurrent callers wait for a free pipeline instead.
// Pipelines are never destroyed (the pool outlives every caller; process exit
// releases the memory), so no HIP call runs during static destruction.
class PipePool {
 public:
  static PipePool &get() {
    static PipePool *p = new PipePool;
    return *p;
  }
  // At most cap_ pipelines per device (several GPUs in one process each get
  // their own: hc_multi_*); a pipeline never moves between devices.
  HostPipe *acquire(int dev) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      for (size_t k = 0; k < idle_.size(); k++)  // an idle pipeline on this device
        if (idle_[k]->dev == dev) return take(k);
      if (live_dev_[dev] < cap_) {
        live_dev_[dev]++;
        live_++;
        auto *p = new HostPipe;
        p->dev = -1;  // initialised on `dev` by the caller
        p->home = dev;
        return p;
      }
      cv_.wait(lk);
    }
  }
  void release(HostPipe *p) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (p->dev < 0) p->dev = p->home;  // (its init failed: it stays this device's)
      idle_.push_back(p);
    }
    cv_.notify_all();
  }
  int live() {
    std::lock_guard<std::mutex> lk(mu_);
    return live_;
  }

 private:
  PipePool() : cap_(std::max(1, env_int("HC_MAX_PIPES", 4))) {}
  HostPipe *take(size_t k) {
    HostPipe *p = idle_[k];
    idle_.erase(idle_.begin() + (long)k);
    return p;
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<HostPipe *> idle_;
  int live_ = 0;
  int live_dev_[kMaxDevices] = {};
  const int cap_;
};

struct PipeLease {  // RAII: one pipeline for one host batch
  HostPipe *p;
  explicit PipeLease(int dev) : p(PipePool::get().acquire(dev)) {}
  ~PipeLease() { PipePool::get().release(p); }
  PipeLease(const PipeLease &) = delete;
  PipeLease &operator=(const PipeLease &) = delete;
};

inline uint64_t blk_off(const uint64_t *off, uint64_t stride, uint64_t i) { return off ? off[i] : i * stride; }
inline uint32_t blk_len(const uint32_t *len, uint32_t ulen, uint64_t i) { return len ? len[i] : ulen; }

bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" of pageable memory
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

thread_local uint64_t t_host_bytes = 0;  // bytes moved by the last host batch (stats)

// Verify on the GPU (CheckBlockIntegrity over the batch): each chunk's kernel
// compares the stored word with the CRC and fills a per-chunk bitmap and lowest
// bad index; retiring chunks merge them here.  No host pass over the caller's
// blocks (one 4-byte read per block at a 4 KiB stride cost 11 % of a 20 GiB
// verify stream when it ran after the batch).
struct HostVerify {
  uint32_t *bitmap = nullptr;  // caller's bitmap, bits set for bad blocks (optional)
  int64_t first_bad = -1;      // lowest bad block (output)
};

// Runs CRCs of host blocks on the GPU; results into crc_out[0..n).  A block
// or message larger than one staging slot (HC_CHUNK_MB, 64 MiB) is hashed on
// its own (oversize): on-disk blocks are 4-16 KiB (utils/config/config.go:137,
// README.md:191,255), but GetCRC / md5.Sum take records of any size.
// md5_out != nullptr: MD5 digests of whole messages instead (row f4; crc_out unused).
constexpr uint64_t kMd5MaxPerChunk = 262144;  // bounds the per-message MD5 workspace of a slot
// hv != nullptr: verify on the GPU (crc_out may be null).  stamp != nullptr:
// each chunk's CRC words are written into stamp + (block offset) as the chunk
// retires (blocks of >= 4 bytes), overlapped with the later chunks' copies.
int host_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
               uint32_t ulen, uint64_t n, uint32_t *crc_out, uint32_t flags, uint8_t *md5_out = nullptr,
               HostVerify *hv = nullptr, uint8_t *stamp = nullptr, int device = -1) {
  const int dev = device >= 0 ? device : default_device();
  int st = init_device(dev);
  if (st != HC_OK) return st;
  PipeLease lease(dev);
  HostPipe &P = *lease.p;
  if ((st = P.init(dev)) != HC_OK) return st;
  DeviceGuard g(dev);
  const bool md5 = md5_out != nullptr;
  const uint64_t maxmsg = md5 ? std::min<uint64_t>(P.maxblk, kMd5MaxPerChunk) : P.maxblk;
  if (md5)
    for (auto &sl : P.slot)
      if (!sl.dmd5 && ((md5_workspace_bytes(maxmsg) &&
                        hipMalloc(reinterpret_cast<void **>(&sl.dtail), md5_workspace_bytes(maxmsg)) != hipSuccess) ||
                       hipMalloc(reinterpret_cast<void **>(&sl.dmd5), maxmsg * 16) != hipSuccess ||
                        hipHostMalloc(reinterpret_cast<void **>(&sl.pin_md5), maxmsg * 16, hipHostMallocDefault) !=
                            hipSuccess))
        return HC_E_NOMEM;
  if (hv)
    for (auto &sl : P.slot)
      if (!sl.dbm && (hipMalloc(reinterpret_cast<void **>(&sl.dbm), (P.maxblk / 32 + 2) * 4) != hipSuccess ||
                      hipMalloc(reinterpret_cast<void **>(&sl.dfb), 8) != hipSuccess ||
                      hipHostMalloc(reinterpret_cast<void **>(&sl.pin_bm), (P.maxblk / 32 + 2) * 4,
                                    hipHostMallocDefault) != hipSuccess ||
                      hipHostMalloc(reinterpret_cast<void **>(&sl.pin_fb), 8, hipHostMallocDefault) != hipSuccess))
        return HC_E_NOMEM;
  const bool want_crc = crc_out || stamp;  // the words come back to the host
  auto mark_bad = [&](uint64_t k) {
    if (hv->bitmap) hv->bitmap[k >> 5] |= 1u << (k & 31);
    if (hv->first_bad < 0 || (int64_t)k < hv->first_bad) hv->first_bad = (int64_t)k;
  };
  auto put_word = [&](uint64_t k, uint32_t c) {
    if (crc_out) crc_out[k] = c;
    if (stamp && blk_len(len, ulen, k) >= HC_CRC_SIZE) std::memcpy(stamp + blk_off(off, stride, k), &c, 4);
  };
  const int copy_threads = (int)std::max<int64_t>(1, knob(kKnobCopyThreads));
  // direct DMA: uniform, densely packed (stride == ulen, 16-B multiple) and already pinned
  const bool direct = !off && !len && stride == ulen && ulen > 0 && (ulen & 15u) == 0 &&
                      (reinterpret_cast<uintptr_t>(base) & 15u) == 0 && is_pinned(base);
  // span DMA: off/len records in pinned memory, in increasing order with small
  // gaps (records packed back to back, e.g. a data component): one H2D copy of
  // the byte span per chunk, no CPU gather
  const bool span_ok = !direct && (off || len) && is_pinned(base);
  uint64_t i = 0, chunks = 0, moved = 0;
  int rc = HC_OK;
  auto retire = [&](Slot &s) -> int {
    if (!s.busy) return HC_OK;
    s.busy = false;
    if (hipEventSynchronize(s.done) != hipSuccess) return HC_E_HIP;
    if (md5) {
      std::memcpy(md5_out + 16 * s.i0, s.pin_md5, s.nb * 16);
      return HC_OK;
    }
    if (crc_out && !stamp)
      std::memcpy(crc_out + s.i0, s.pin_crc, s.nb * 4);
    else if (want_crc)
      for (uint64_t k = 0; k < s.nb; k++) put_word(s.i0 + k, s.pin_crc[k]);
    if (hv && *s.pin_fb < s.nb)  // something failed in this chunk: merge its bits
      for (uint64_t w = 0; w < (s.nb + 31) / 32; w++)
        for (uint32_t m = s.pin_bm[w]; m; m &= m - 1) mark_bad(s.i0 + 32 * w + (uint32_t)__builtin_ctz(m));
    return HC_OK;
  };
  // A block or message larger than a staging slot (records are uint32-sized):
  // its own device buffer, copied and hashed synchronously on the slot's stream.
  auto oversize = [&](Slot &s, uint64_t k) -> int {
    const uint64_t o = blk_off(off, stride, k);
    const uint32_t l = blk_len(len, ulen, k);
    uint8_t *d = nullptr;
    int r = HC_OK;
    if (hipMallocAsync(reinterpret_cast<void **>(&d), (size_t)l + 16, s.stream) != hipSuccess) return HC_E_NOMEM;
    if (hipMemcpyAsync(d, base + o, l, hipMemcpyHostToDevice, s.stream) != hipSuccess) r = HC_E_HIP;
    if (r == HC_OK && md5) {
      if (launch_md5(d, nullptr, nullptr, l, l, 1, s.dtail, s.dmd5, g_dev[dev].cus, s.stream) != hipSuccess ||
          hipMemcpyAsync(s.pin_md5, s.dmd5, 16, hipMemcpyDeviceToHost, s.stream) != hipSuccess)
        r = HC_E_HIP;
    } else if (r == HC_OK) {
      r = dispatch(dev, d, nullptr, nullptr, l, l, 1, s.dcrc, nullptr, nullptr, flags, s.stream, l);
      if (r == HC_OK && hipMemcpyAsync(s.pin_crc, s.dcrc, 4, hipMemcpyDeviceToHost, s.stream) != hipSuccess)
        r = HC_E_HIP;
    }
    if (hipFreeAsync(d, s.stream) != hipSuccess && r == HC_OK) r = HC_E_HIP;
    if (hipStreamSynchronize(s.stream) != hipSuccess && r == HC_OK) r = HC_E_HIP;
    if (r == HC_OK) {
      if (md5) {
        std::memcpy(md5_out + 16 * k, s.pin_md5, 16);
      } else {
        put_word(k, s.pin_crc[0]);
        if (hv) {  // one block on its own: compare here (l > 64 MiB >= 4)
          uint32_t stored;
          std::memcpy(&stored, base + o, 4);
          if (stored != s.pin_crc[0]) mark_bad(k);
        }
      }
      moved += l;
    }
    return r;
  };
  while (i < n && rc == HC_OK) {
    Slot &s = P.slot[chunks % kSlots];
    if ((rc = retire(s)) != HC_OK) break;
    uint64_t j = i, pos = 0;
    bool packed_uniform;
    uint8_t *dsrc = s.dbuf;  // the chunk's device copy
    uint32_t l0 = blk_len(len, ulen, i);
    if (direct) {
      if (ulen > P.chunk) {  // a block larger than a staging slot: on its own
        if ((rc = oversize(s, i)) != HC_OK) break;
        i++;
        continue;
      }
      j = std::min<uint64_t>(n, i + P.chunk / ulen);
      j = std::min<uint64_t>(j, i + maxmsg);
      pos = (j - i) * (uint64_t)ulen;
      if (hipMemcpyAsync(s.dbuf, base + i * stride, pos, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
        rc = HC_E_HIP;
        break;
      }
      packed_uniform = true;
    } else if (span_ok && (s.dspan || hipMalloc(reinterpret_cast<void **>(&s.dspan), P.span) == hipSuccess) && [&] {
                 // plan [i, j) as one span; keep its 16-B phase when the bytes
                 // before the first block belong to the caller's buffer
                 const uint64_t lo = blk_off(off, stride, i);
                 uint64_t ph = (reinterpret_cast<uintptr_t>(base) + lo) & 15u;
                 if (lo < ph) ph = 0;
                 uint64_t hi = lo, payload = 0;
                 while (j < n && j - i < maxmsg) {
                   const uint64_t o = blk_off(off, stride, j);
                   const uint32_t l = blk_len(len, ulen, j);
                   if (o < hi && j > i) break;  // overlap or out of order: end the span
                   const uint64_t nhi = std::max<uint64_t>(hi, o + l);
                   if (nhi - lo + ph > P.span) break;
                   s.pin_off[j - i] = o - lo + ph;
                   s.pin_len[j - i] = l;
                   hi = nhi;
                   payload += l;
                   j++;
                 }
                 pos = hi - lo + ph;
                 if (j == i || pos > payload + payload / 4 + (64u << 10)) {  // gaps: gather instead
                   j = i;
                   pos = 0;
                   return false;
                 }
                 dsrc = s.dspan;
                 return hipMemcpyAsync(s.dspan, base + lo - ph, pos, hipMemcpyHostToDevice, s.stream) == hipSuccess;
               }()) {
      const uint64_t nb = j - i;
      packed_uniform = false;
      if (hipMemcpyAsync(s.doff, s.pin_off, nb * 8, hipMemcpyHostToDevice, s.stream) != hipSuccess ||
          hipMemcpyAsync(s.dlen, s.pin_len, nb * 4, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
        rc = HC_E_HIP;
        break;
      }
    } else {
      if (j != i) {  // the span copy failed to enqueue
        rc = HC_E_HIP;
        break;
      }
      // plan the chunk: blocks [i, j) packed at 16-B aligned offsets, or back
      // to back when the source is one contiguous run of equal blocks (then
      // each gather thread copies one span; unaligned blocks go to k_crc_any)
      bool uniform = true;
      const bool contig = !off && !len && stride == ulen;
      while (j < n && j - i < maxmsg) {
        const uint32_t l = blk_len(len, ulen, j);
        const uint64_t need = contig ? pos + l : (pos + l + 15) & ~uint64_t(15);
        if (need > P.chunk) break;
        s.pin_off[j - i] = pos;
        s.pin_len[j - i] = l;
        uniform = uniform && l == l0;
        pos = need;
        j++;
      }
      if (j == i) {  // one block/message larger than a staging slot: on its own
        if ((rc = oversize(s, i)) != HC_OK) break;
        i++;
        continue;
      }
      const uint64_t nb = j - i;
      // gather into pinned staging on copy_threads threads
      const int th = (int)std::min<uint64_t>((uint64_t)copy_threads, std::max<uint64_t>(1, pos >> 22));
      // streamed stores into staging (only the DMA engine reads it): neutral for
      // block batches, +4-10 % for WAL replay, whose record copy-out competes
      // for host memory bandwidth (profiles/r2/host_gather/)
      parallel_for(th, [&](int t) {
        const uint64_t a = nb * t / th, b = nb * (t + 1) / th;
        // contiguous source AND contiguous staging (pin_off[k] = k*ulen): one copy per thread
        if (contig) {
          if (b > a) copy_nt(s.pin + s.pin_off[a], base + (i + a) * stride, (b - a) * (uint64_t)ulen);
        } else {
          for (uint64_t k = a; k < b; k++)
            copy_nt(s.pin + s.pin_off[k], base + blk_off(off, stride, i + k), s.pin_len[k]);
        }
        _mm_sfence();  // streamed staging bytes are visible to the DMA engine
      });
      packed_uniform = uniform && (l0 & 15u) == 0;  // then off = k*l0
      if (hipMemcpyAsync(s.dbuf, s.pin, pos, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
        rc = HC_E_HIP;
        break;
      }
      if (!packed_uniform &&
          (hipMemcpyAsync(s.doff, s.pin_off, nb * 8, hipMemcpyHostToDevice, s.stream) != hipSuccess ||
           hipMemcpyAsync(s.dlen, s.pin_len, nb * 4, hipMemcpyHostToDevice, s.stream) != hipSuccess)) {
        rc = HC_E_HIP;
        break;
      }
    }
    const uint64_t nb = j - i;
    if (md5) {
      const bool u = packed_uniform;
      if (launch_md5(dsrc, u ? nullptr : s.doff, u ? nullptr : s.dlen, l0, l0, nb, s.dtail, s.dmd5,
                     g_dev[dev].cus, s.stream) != hipSuccess ||
          hipMemcpyAsync(s.pin_md5, s.dmd5, nb * 16, hipMemcpyDeviceToHost, s.stream) != hipSuccess) {
        rc = HC_E_HIP;
        break;
      }
      t_last = hc_launch_info{"k_md5", 0, nb, pos, 0, 256, 0};
    } else {
      uint32_t *dbm = hv ? s.dbm : nullptr;
      int64_t *dfb = hv ? reinterpret_cast<int64_t *>(s.dfb) : nullptr;
      if (hv && launch_verify_prepare(s.dbm, s.dfb, nb, s.stream) != hipSuccess) {
        rc = HC_E_HIP;
        break;
      }
      rc = packed_uniform
               ? dispatch(dev, dsrc, nullptr, nullptr, l0, l0, nb, s.dcrc, dbm, dfb, flags, s.stream, pos)
               : dispatch(dev, dsrc, s.doff, s.dlen, 0, 0, nb, s.dcrc, dbm, dfb, flags, s.stream, pos);
      if (rc != HC_OK) break;
      if ((want_crc && hipMemcpyAsync(s.pin_crc, s.dcrc, nb * 4, hipMemcpyDeviceToHost, s.stream) != hipSuccess) ||
          (hv && (hipMemcpyAsync(s.pin_fb, s.dfb, 8, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
                  hipMemcpyAsync(s.pin_bm, s.dbm, (nb + 31) / 32 * 4, hipMemcpyDeviceToHost, s.stream) !=
                      hipSuccess))) {
        rc = HC_E_HIP;
        break;
      }
    }
    if (hipEventRecord(s.done, s.stream) != hipSuccess) {
      rc = HC_E_HIP;
      break;
    }
    s.i0 = i;
    s.nb = nb;
    s.busy = true;
    moved += pos;
    i = j;
    chunks++;
  }
  for (auto &s : P.slot) {
    int r = retire(s);
    if (rc == HC_OK) rc = r;
  }
  t_host_bytes = moved;
  return rc;
}

}  // namespace

// ===========================================================================
// C ABI
extern "C" {

const char *hc_strerror(int code) {
  switch (code) {
    case HC_OK: return "";
    case HC_ERR_INVALID_BLOCK: return "invalid block data";
    case HC_ERR_CRC_MISMATCH: return "CRC mismatch in block";
    case HC_ERR_TOO_SHORT: return "data is too short to contain a complete block";
    case HC_ERR_WAL_FRAGMENT_TYPE: return "unknown fragment type";
    case HC_ERR_WAL_TRUNCATED: return "WAL fragment overruns its block";
    case HC_E_ARG: return "hundcrc: invalid argument";
    case HC_E_HIP: return "hundcrc: HIP runtime error";
    case HC_E_NODEV: return "hundcrc: no gfx950 device available (the GPU path never falls back to the CPU)";
    case HC_E_NOMEM: return "hundcrc: device or pinned allocation failed";
    case HC_E_LAYOUT: return "hundcrc: device batch violates the layout contract";
    default: return "hundcrc: unknown error";
  }
}

const char *hc_version(void) { return "hundcrc 0.1.0 (gfx950)"; }

int hc_device_count(void) {
  int n = device_count_raw(), good = 0;
  for (int i = 0; i < n && i < kMaxDevices; i++) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess &&
        std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
      good++;
  }
  return good;
}

// ---- drop-ins ---------------------------------------------------------------
uint32_t hc_crc32_ieee(const uint8_t *p, size_t n) {
  if (n == 0) return 0;
  if (force_gpu() && n <= 0xFFFFFFFFu) {
    // HC_FORCE_GPU is a test mode: a broken GPU path must not pass on the CPU.
    // GetCRC has no error channel (crc_util.go:15), so report and abort.
    uint64_t o = 0;
    uint32_t l = (uint32_t)n, c = 0;
    const int rc = host_batch(p, &o, &l, 0, 0, 1, &c, kFlagMessages);
    if (rc != HC_OK) {
      std::fprintf(stderr, "hundcrc: HC_FORCE_GPU GetCRC failed: %s\n", hc_strerror(rc));
      std::abort();
    }
    return c;
  }
  return hc::cpu_crc32_update(0, p, n);
}

int hc_add_crc_block(uint8_t *p, size_t n) {
  if (n < HC_CRC_SIZE) return HC_OK;  // crc_util.go:22-24
  if (!p) return HC_E_ARG;
  uint32_t c;
  if (force_gpu() && n <= 0xFFFFFFFFu) {
    uint64_t o = 0;
    uint32_t l = (uint32_t)n;
    int rc = host_batch(p, &o, &l, 0, 0, 1, &c, 0);
    if (rc != HC_OK) return rc;
  } else {
    c = hc::cpu_crc32_update(0, p + HC_CRC_SIZE, n - HC_CRC_SIZE);
  }
  std::memcpy(p, &c, 4);  // binary.LittleEndian.PutUint32 (crc_util.go:30)
  return HC_OK;
}

size_t hc_add_crcs_size(size_t n) { return (n + kPayloadPerBlock - 1) / kPayloadPerBlock * HC_BLOCK_SIZE; }

size_t hc_add_crcs(const uint8_t *src, size_t n, uint8_t *dst, size_t dst_cap) {
  const size_t out = hc_add_crcs_size(n);
  if (out > dst_cap || (n && (!src || !dst))) return (size_t)-1;
  const size_t nb = out / HC_BLOCK_SIZE;
  const size_t nfull = n / kPayloadPerBlock;  // blocks whose 4092 payload bytes all come from src
  // framing: zeroed 4096-byte blocks, payload at [4:] (crc_util.go:48-60)
  auto frame = [&](size_t a, size_t b) {
    for (size_t k = a; k < b; k++) {
      uint8_t *blk = dst + k * HC_BLOCK_SIZE;
      const size_t s = k * kPayloadPerBlock, e = std::min(n, s + kPayloadPerBlock);
      std::memset(blk, 0, HC_CRC_SIZE);
      std::memcpy(blk + HC_CRC_SIZE, src + s, e - s);
      if (e - s < kPayloadPerBlock) std::memset(blk + HC_CRC_SIZE + (e - s), 0, kPayloadPerBlock - (e - s));
    }
  };

  // CRCs: one GPU batch for multi-block outputs, host for small ones.
  // AddCRCsToData cannot fail in Go (crc_util.go:41-64), so a GPU batch that
  // does not complete -- no gfx950 (HC_E_NODEV), a device or pinned allocation
  // failure (HC_E_NOMEM), a HIP runtime error (HC_E_HIP) -- is finished on the
  // host path below (hc_cpu.cpp, product code) from the already framed dst,
  // and counted in hc_stats.  Only HC_FORCE_GPU (test mode) returns the error.
  // HC_INJECT_FAIL=add_crcs[:nomem] simulates a failing GPU batch (tests).
  const size_t gpu_min = (size_t)knob(kKnobAddCrcsGpuMin);  // hc_debug_set: tools/crossover.py
  bool on_gpu = false;
  if (nb >= gpu_min || (force_gpu() && nb > 0)) {
    // The CRC of block k is ChecksumIEEE(src[4092k : 4092k+4092]) for every
    // full block, so the GPU batch reads the SOURCE payload (4092-byte
    // messages; one span DMA per chunk when src is pinned) while
    // HC_COPY_THREADS threads frame dst: the two overlap instead of framing
    // first and reading dst back.  The ragged last block (zero-padded) is
    // hashed on the host after framing.
    // framing tasks: HC_COPY_THREADS (8), one per MiB of output at most
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max<int64_t>(1, knob(kKnobCopyThreads)), nb >> 8));
    std::vector<uint32_t> crc(nfull);
    int rc = HC_OK;
    // (plain stores: streamed framing measured 10-35 % slower, profiles/r2/addcrcs/)
    // task 0 is the GPU batch, so the caller starts it at once
    parallel_for(T + 1, [&](int t) {
      if (t > 0) {
        frame(nb * (t - 1) / T, nb * t / T);
        return;
      }
      if (!nfull) return;
      if (const int inj = injected_failure(kInjectAddCrcs)) {
        rc = inj;
        return;
      }
      if (is_pinned(src)) {  // span DMA wants explicit off/len
        std::vector<uint64_t> o(nfull);
        std::vector<uint32_t> l(nfull, (uint32_t)kPayloadPerBlock);
        for (size_t k = 0; k < nfull; k++) o[k] = k * kPayloadPerBlock;
        rc = host_batch(src, o.data(), l.data(), 0, 0, nfull, crc.data(), kFlagMessages);
      } else {
        rc = host_batch(src, nullptr, nullptr, kPayloadPerBlock, (uint32_t)kPayloadPerBlock, nfull, crc.data(),
                        kFlagMessages);
      }
    });
    if (rc == HC_OK) {
      parallel_for(T, [&](int t) {  // the words into the framed blocks
        for (size_t k = nfull * t / T, e = nfull * (t + 1) / T; k < e; k++)
          std::memcpy(dst + k * HC_BLOCK_SIZE, &crc[k], 4);
      });
      for (size_t k = nfull; k < nb; k++) {  // the ragged last block
        uint8_t *blk = dst + k * HC_BLOCK_SIZE;
        const uint32_t c = hc::cpu_crc32_update(0, blk + HC_CRC_SIZE, kPayloadPerBlock);
        std::memcpy(blk, &c, 4);
      }
      on_gpu = true;
      g_stats.add_crcs_gpu.fetch_add(1, std::memory_order_relaxed);
    } else if (force_gpu() || !gpu_batch_failure(rc)) {
      return (size_t)-1;
    } else if (rc == HC_E_NODEV) {
      g_stats.add_crcs_host_nodev.fetch_add(1, std::memory_order_relaxed);
    } else {
      count_fallback(g_stats.add_crcs_gpu_fallback, rc);
    }
  } else {
    frame(0, nb);
    g_stats.add_crcs_host_small.fetch_add(1, std::memory_order_relaxed);
  }
  if (!on_gpu) {
    for (size_t b = 0; b < nb; b++) {
      uint8_t *blk = dst + b * HC_BLOCK_SIZE;
      const uint32_t c = hc::cpu_crc32_update(0, blk + HC_CRC_SIZE, kPayloadPerBlock);
      std::memcpy(blk, &c, 4);
    }
  }
  return out;
}

uint64_t hc_size_after_crcs(uint64_t n) {
  // int(math.Ceil(float64(n) / float64(4092))) -- crc_util.go:70-71
  const int64_t nb = (int64_t)std::ceil((double)n / (double)kPayloadPerBlock);
  return n + (uint64_t)nb * HC_CRC_SIZE;
}

uint64_t hc_size_without_crcs(uint64_t n) {
  // uint64(math.Ceil(float64(n) / float64(4096))) -- crc_util.go:80; wraps for 0<n<4
  const uint64_t nb = (uint64_t)std::ceil((double)n / (double)HC_BLOCK_SIZE);
  return n - nb * HC_CRC_SIZE;
}

int hc_check_block(const uint8_t *p, size_t n) {
  if (n < HC_CRC_SIZE) return HC_ERR_INVALID_BLOCK;  // crc_util.go:89-91
  uint32_t stored;
  std::memcpy(&stored, p, 4);
  uint32_t c;
  if (force_gpu() && n <= 0xFFFFFFFFu) {
    uint64_t o = 0;
    uint32_t l = (uint32_t)n;
    int rc = host_batch(p, &o, &l, 0, 0, 1, &c, 0);
    if (rc != HC_OK) return rc;
  } else {
    c = hc::cpu_crc32_update(0, p + HC_CRC_SIZE, n - HC_CRC_SIZE);
  }
  return stored == c ? HC_OK : HC_ERR_CRC_MISMATCH;
}

int hc_fix_last_block(uint8_t *p, size_t n) {
  if (n < HC_BLOCK_SIZE) return HC_ERR_TOO_SHORT;  // crc_util.go:107-109
  const size_t complete = n / HC_BLOCK_SIZE;
  return hc_add_crc_block(p + (complete - 1) * HC_BLOCK_SIZE, HC_BLOCK_SIZE);
}

// ---- host-resident batches ---------------------------------------------------
int hc_crc32_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                    uint32_t ulen, uint64_t nblocks, uint32_t *crc_out) {
  if (nblocks == 0) return HC_OK;
  if (!base || !crc_out) return HC_E_ARG;
  return host_batch(base, off, len, stride, ulen, nblocks, crc_out, 0);
}

int hc_crc32_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                      uint32_t *crc_out) {
  if (n == 0) return HC_OK;
  if (!base || !off || !len || !crc_out) return HC_E_ARG;
  return host_batch(base, off, len, 0, 0, n, crc_out, kFlagMessages);
}

int hc_md5_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out16) {
  if (n == 0) return HC_OK;
  if (!base || !off || !len || !out16) return HC_E_ARG;
  return host_batch(base, off, len, 0, 0, n, nullptr, 0, out16);
}

int hc_verify_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                     uint32_t ulen, uint64_t nblocks, uint32_t *bad_bitmap, int64_t *first_bad) {
  if (first_bad) *first_bad = -1;
  if (bad_bitmap) std::memset(bad_bitmap, 0, ((nblocks + 31) / 32) * 4);
  if (nblocks == 0) return HC_OK;
  if (!base) return HC_E_ARG;
  // the kernels compare on the GPU (len < 4 is always bad there, as in
  // crc_util.go:89-91); the host only merges the per-chunk bitmaps
  HostVerify hv;
  hv.bitmap = bad_bitmap;
  int rc = host_batch(base, off, len, stride, ulen, nblocks, nullptr, 0, nullptr, &hv);
  if (rc != HC_OK) return rc;
  if (hv.first_bad < 0) return HC_OK;
  if (first_bad) *first_bad = hv.first_bad;
  return blk_len(len, ulen, (uint64_t)hv.first_bad) < HC_CRC_SIZE ? HC_ERR_INVALID_BLOCK : HC_ERR_CRC_MISMATCH;
}

int hc_stamp_blocks(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                    uint32_t ulen, uint64_t nblocks) {
  if (nblocks == 0) return HC_OK;
  if (!base) return HC_E_ARG;
  // words written into the caller's blocks as each chunk retires
  return host_batch(base, off, len, stride, ulen, nblocks, nullptr, 0, nullptr, nullptr, base);
}

// ---- several GPUs in one process ---------------------------------------------
int hc_shard_plan(uint64_t nblocks, const uint32_t *len, int ndev, uint64_t *bounds) {
  if (ndev < 1 || ndev > kMaxDevices || !bounds) return HC_E_ARG;
  bounds[0] = 0;
  bounds[ndev] = nblocks;
  if (!len) {  // shard.index_range: n*d/ndev
    for (int d = 1; d < ndev; d++) bounds[d] = (uint64_t)((unsigned __int128)nblocks * (unsigned)d / (unsigned)ndev);
    return HC_OK;
  }
  // shard.byte_balanced_bounds: the first block whose prefix sum (bytes of the
  // blocks before it) reaches total*d/ndev
  unsigned __int128 total = 0;
  for (uint64_t i = 0; i < nblocks; i++) total += len[i];
  uint64_t i = 0;
  unsigned __int128 csum = 0;  // bytes of blocks [0, i)
  for (int d = 1; d < ndev; d++) {
    const unsigned __int128 target = total * (unsigned)d / (unsigned)ndev;
    while (i < nblocks && csum < target) csum += len[i++];
    bounds[d] = i;
  }
  return HC_OK;
}

}  // extern "C"

namespace {
// Runs fn(d, lo, hi, device) for every shard d on its own thread (the caller's
// for shard 0) after checking the plan; returns the first failing shard's code.
template <class F>
int multi_run(uint64_t nblocks, const uint32_t *len, int ndev, const int *devices, const uint64_t *bounds_in,
              F &&fn) {
  if (ndev < 1 || ndev > kMaxDevices || !devices) return HC_E_ARG;
  std::vector<uint64_t> bounds(ndev + 1);
  if (bounds_in) {
    std::copy(bounds_in, bounds_in + ndev + 1, bounds.begin());
    if (bounds[0] != 0 || bounds[ndev] != nblocks) return HC_E_ARG;
    for (int d = 0; d < ndev; d++)
      if (bounds[d] > bounds[d + 1]) return HC_E_ARG;
  } else if (hc_shard_plan(nblocks, len, ndev, bounds.data()) != HC_OK) {
    return HC_E_ARG;
  }
  for (int d = 0; d < ndev; d++) {
    const int st = init_device(devices[d]);
    if (st != HC_OK) return st;
  }
  std::vector<int> rc(ndev, HC_OK);
  parallel_for(ndev, [&](int d) {
    if (bounds[d + 1] > bounds[d]) rc[d] = fn(d, bounds[d], bounds[d + 1], devices[d]);
  });
  for (int d = 0; d < ndev; d++)
    if (rc[d] != HC_OK) return rc[d];
  return HC_OK;
}
}  // namespace

extern "C" {

int hc_multi_crc32_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                          uint32_t ulen, uint64_t nblocks, uint32_t *crc_out, int ndev, const int *devices,
                          const uint64_t *bounds) {
  if (nblocks == 0) return HC_OK;
  if (!base || !crc_out) return HC_E_ARG;
  return multi_run(nblocks, len, ndev, devices, bounds, [&](int, uint64_t lo, uint64_t hi, int dev) {
    return host_batch(off ? base : base + lo * stride, off ? off + lo : nullptr, len ? len + lo : nullptr, stride,
                      ulen, hi - lo, crc_out + lo, 0, nullptr, nullptr, nullptr, dev);
  });
}

int hc_multi_verify_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                           uint32_t ulen, uint64_t nblocks, uint32_t *bad_bitmap, int64_t *first_bad, int ndev,
                           const int *devices, const uint64_t *bounds) {
  if (first_bad) *first_bad = -1;
  if (bad_bitmap) std::memset(bad_bitmap, 0, ((nblocks + 31) / 32) * 4);
  if (nblocks == 0) return HC_OK;
  if (!base || ndev < 1 || ndev > kMaxDevices) return HC_E_ARG;
  // each shard verifies into a bitmap of its own (its blocks from bit 0)
  std::vector<std::vector<uint32_t>> bm(ndev);
  std::vector<int64_t> fb(ndev, -1);
  std::vector<uint64_t> los(ndev, 0);
  const int rc = multi_run(nblocks, len, ndev, devices, bounds, [&](int d, uint64_t lo, uint64_t hi, int dev) {
    HostVerify hv;
    if (bad_bitmap) {
      bm[d].assign((hi - lo + 31) / 32, 0);
      hv.bitmap = bm[d].data();
    }
    los[d] = lo;
    const int r = host_batch(off ? base : base + lo * stride, off ? off + lo : nullptr, len ? len + lo : nullptr,
                             stride, ulen, hi - lo, nullptr, 0, nullptr, &hv, nullptr, dev);
    fb[d] = hv.first_bad;
    return r;
  });
  if (rc != HC_OK) return rc;
  int64_t first = -1;
  for (int d = 0; d < ndev; d++) {
    if (fb[d] < 0) continue;
    const int64_t g = (int64_t)los[d] + fb[d];
    if (first < 0 || g < first) first = g;
    for (uint64_t w = 0; w < bm[d].size(); w++)
      for (uint32_t m = bm[d][w]; m; m &= m - 1) {
        const uint64_t k = los[d] + 32 * w + (uint32_t)__builtin_ctz(m);
        bad_bitmap[k >> 5] |= 1u << (k & 31);
      }
  }
  if (first < 0) return HC_OK;
  if (first_bad) *first_bad = first;
  return blk_len(len, ulen, (uint64_t)first) < HC_CRC_SIZE ? HC_ERR_INVALID_BLOCK : HC_ERR_CRC_MISMATCH;
}

int hc_multi_stamp_blocks(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t ulen,
                          uint64_t nblocks, int ndev, const int *devices, const uint64_t *bounds) {
  if (nblocks == 0) return HC_OK;
  if (!base) return HC_E_ARG;
  return multi_run(nblocks, len, ndev, devices, bounds, [&](int, uint64_t lo, uint64_t hi, int dev) {
    uint8_t *b = off ? base : base + lo * stride;
    return host_batch(b, off ? off + lo : nullptr, len ? len + lo : nullptr, stride, ulen, hi - lo, nullptr, 0,
                      nullptr, nullptr, b, dev);
  });
}

// ---- device-resident batches ---------------------------------------------------
int hc_dev_crc32_blocks(int device, const void *base, const uint64_t *off, const uint32_t *len,
                        uint64_t stride, uint32_t ulen, uint64_t nblocks, uint32_t *crc_out,
                        uint32_t *bad_bitmap, int64_t *first_bad, uint32_t flags, void *stream) {
  if (nblocks == 0) return HC_OK;
  if (!base) return HC_E_ARG;
  if (bad_bitmap && !first_bad) return HC_E_ARG;
  if ((flags & HC_F_MESSAGES) && (first_bad || (flags & HC_F_STAMP))) return HC_E_ARG;
  int st = init_device(device);
  if (st != HC_OK) return st;
  DeviceGuard g(device);
  uint64_t bytes = (!off && !len) ? nblocks * (uint64_t)ulen : 0;
  return dispatch(device, static_cast<const uint8_t *>(base), off, len, stride, ulen, nblocks, crc_out,
                  bad_bitmap, first_bad, flags, static_cast<hipStream_t>(stream), bytes, true);
}

int hc_dev_multi_crc32_blocks(const hc_dev_shard *shards, int nshards, uint32_t flags) {
  if (nshards < 0 || (nshards > 0 && !shards)) return HC_E_ARG;
  for (int k = 0; k < nshards; k++) {
    const hc_dev_shard &h = shards[k];
    const int rc = hc_dev_crc32_blocks(h.device, h.base, h.off, h.len, h.stride, h.ulen, h.nblocks, h.crc_out,
                                       h.bad_bitmap, h.first_bad, flags, h.stream);
    if (rc != HC_OK) return rc;
  }
  return HC_OK;
}

uint64_t hc_read_blocks_touched(uint32_t block_size, uint64_t start_offset, uint64_t size) {
  const uint64_t B = block_size;
  if (B <= HC_CRC_SIZE || size == 0) return 0;
  uint64_t boff = start_offset % B;
  if (boff < HC_CRC_SIZE) boff = HC_CRC_SIZE;  // block_manager.go:198-201
  const uint64_t first = B - boff;              // payload bytes of the first block
  return size <= first ? 1 : 1 + (size - first + (B - 5)) / (B - 4);
}

int hc_read_from_disk_v(const uint8_t *blocks, uint64_t avail, uint32_t block_size, uint64_t start_offset,
                        uint64_t size, uint32_t *verified, uint8_t *out, uint64_t *final_offset, int64_t *bad_block,
                        uint64_t *hashed) {
  if (bad_block) *bad_block = -1;
  if (hashed) *hashed = 0;
  const uint64_t B = block_size;
  if (B <= HC_CRC_SIZE || (size && !out) || (avail && !blocks)) return HC_E_ARG;
  uint64_t boff = start_offset % B;
  if (boff < HC_CRC_SIZE) boff = HC_CRC_SIZE;  // block_manager.go:198-201
  // blocks touched by the loop at :207-235
  const uint64_t k = hc_read_blocks_touched(block_size, start_offset, size);
  auto known_good = [&](uint64_t i) { return verified && ((verified[i >> 5] >> (i & 31)) & 1u); };
  auto mark = [&](uint64_t i) {
    if (verified) verified[i >> 5] |= 1u << (i & 31);
  };
  // Verify every touched block the caller has not already verified (its cache's
  // verified bit, lru_cache.go:51-65 entries filled by ReadBlock :91-97) in ONE
  // batch (a9); the first failing block in order is the one the Go loop stops at.
  const uint64_t nfull = std::min<uint64_t>(k, avail / B);
  std::vector<uint64_t> todo;
  todo.reserve(nfull);
  for (uint64_t i = 0; i < nfull; i++)
    if (!known_good(i)) todo.push_back(i);
  int64_t bad = -1;
  // append blockData[blockOffset : blockOffset+bytesToRead] of blocks [a, b)
  // (:221-231); block i's output position is known in closed form: the first
  // block gives B - boff bytes, every later one B - 4, capped at `size`
  const uint64_t boff0 = boff, first_take = B - boff0;
  auto produced_before = [&](uint64_t i) -> uint64_t {
    return i == 0 ? 0 : std::min<uint64_t>(size, first_take + (i - 1) * (B - HC_CRC_SIZE));
  };
  auto copy_out = [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; i++) {
      const uint64_t produced = produced_before(i);
      const uint64_t bo = i == 0 ? boff0 : HC_CRC_SIZE;
      const uint64_t take = std::min<uint64_t>(size - produced, B - bo);
      if (take == 0) continue;  // (out may be null when size == 0)
      const uint64_t o = i * B + bo;
      // bytes past `avail` are zeros
      const uint64_t have = o >= avail ? 0 : std::min<uint64_t>(take, avail - o);
      if (have) std::memcpy(out + produced, blocks + o, have);
      if (have < take) std::memset(out + produced + have, 0, take - have);
    }
  };
  bool copied = false, on_gpu = false;
  const uint64_t gpu_min = (uint64_t)knob(kKnobReadGpuMin);  // hc_debug_set: tools/crossover.py
  const uint64_t nt = todo.size();
  std::vector<uint8_t> ok(nt, 0);
  if (nt && (nt >= gpu_min || force_gpu()) && B <= 0xFFFFFFFFu) {
    // verified on the GPU: bit j of `badj` = todo[j] failed
    std::vector<uint32_t> badj((nt + 31) / 32, 0);
    HostVerify hv;
    hv.bitmap = badj.data();
    // the copy-out runs on HC_COPY_THREADS threads while the batch verifies;
    // on a CRC failure `out` is left unspecified (Go returns no data)
    // copy-out tasks: HC_COPY_THREADS (8), one per MiB of blocks at most; task 0
    // is the GPU batch, so the caller starts it at once
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max<int64_t>(1, knob(kKnobCopyThreads)),
                                                                 k * B >> 20));
    int rc = HC_OK;
    parallel_for(T + 1, [&](int t) {
      if (t > 0) {
        copy_out(k * (t - 1) / T, k * t / T);
        return;
      }
      if ((rc = injected_failure(kInjectReadFromDisk)) != HC_OK) return;
      if (nt == nfull) {  // nothing masked: one uniform batch
        rc = host_batch(blocks, nullptr, nullptr, B, (uint32_t)B, nt, nullptr, 0, nullptr, &hv);
      } else {
        std::vector<uint64_t> off(nt);
        std::vector<uint32_t> len(nt, (uint32_t)B);
        for (uint64_t j = 0; j < nt; j++) off[j] = todo[j] * B;
        rc = host_batch(blocks, off.data(), len.data(), 0, 0, nt, nullptr, 0, nullptr, &hv);
      }
    });
    copied = true;
    if (rc == HC_OK) {
      for (uint64_t j = 0; j < nt; j++) ok[j] = !((badj[j >> 5] >> (j & 31)) & 1u);
      on_gpu = true;
      g_stats.read_gpu.fetch_add(1, std::memory_order_relaxed);
    } else if (force_gpu() || !gpu_batch_failure(rc)) {
      return rc;
    } else {  // ReadFromDisk fails only on I/O or a CRC mismatch: finish on the host path
      count_fallback(g_stats.read_gpu_fallback, rc);
    }
  }
  if (!on_gpu) {
    for (uint64_t j = 0; j < nt; j++) {
      const uint8_t *blk = blocks + todo[j] * B;
      uint32_t stored;
      std::memcpy(&stored, blk, 4);
      ok[j] = stored == hc::cpu_crc32_update(0, blk + HC_CRC_SIZE, B - HC_CRC_SIZE);
    }
  }
  for (uint64_t j = 0; j < nt; j++) {
    if (ok[j]) {
      mark(todo[j]);
    } else if (bad < 0) {
      bad = (int64_t)todo[j];
    }
  }
  uint64_t nhashed = nt;
  std::vector<uint8_t> tailbuf;
  if (bad < 0 && nfull < k) {
    // blocks past `avail`: ReadBlock returns a zero-extended short read (:130-146)
    tailbuf.assign(B, 0);
    for (uint64_t i = nfull; i < k && bad < 0; i++) {
      if (known_good(i)) continue;
      std::fill(tailbuf.begin(), tailbuf.end(), 0);
      const uint64_t o = i * B;
      if (o < avail) std::memcpy(tailbuf.data(), blocks + o, std::min<uint64_t>(B, avail - o));
      uint32_t stored;
      std::memcpy(&stored, tailbuf.data(), 4);
      nhashed++;
      if (stored != hc::cpu_crc32_update(0, tailbuf.data() + HC_CRC_SIZE, B - HC_CRC_SIZE)) bad = (int64_t)i;
    }
  }
  if (hashed) *hashed = nhashed;
  if (bad >= 0) {
    if (bad_block) *bad_block = bad;
    return HC_ERR_CRC_MISMATCH;
  }
  if (!copied) copy_out(0, k);
  if (final_offset) *final_offset = hc_size_after_crcs(hc_size_without_crcs(start_offset) + size);  // :237-239
  return HC_OK;
}

int hc_read_from_disk(const uint8_t *blocks, uint64_t avail, uint32_t block_size, uint64_t start_offset,
                      uint64_t size, uint8_t *out, uint64_t *final_offset, int64_t *bad_block) {
  return hc_read_from_disk_v(blocks, avail, block_size, start_offset, size, nullptr, out, final_offset, bad_block,
                             nullptr);
}

int hc_dev_add_crcs(int device, const void *src, uint64_t n, void *dst, uint32_t *crc_out, void *stream) {
  if (n == 0) return HC_OK;  // Go returns an empty slice
  if (!src || !dst) return HC_E_ARG;
  if ((reinterpret_cast<uintptr_t>(dst) & 15u) != 0) return HC_E_LAYOUT;
  const uint64_t nblk = (n + kPayloadPerBlock - 1) / kPayloadPerBlock;
  // k_frame: edges + one interior block per wave
  const uint64_t wgs = 1 + (nblk > 2 ? kFrameSpread * ((nblk - 2 + 4 * kFrameSpread - 1) / (4 * kFrameSpread)) : 0);
  if (wgs > kMaxGridWgs) return HC_E_ARG;  // over 2^32 work-items (~68 TB of payload)
  int st = init_device(device);
  if (st != HC_OK) return st;
  DeviceGuard g(device);
  DeviceState &d = g_dev[device];
  const int grid = (int)wgs;
  hc_launch_info info{"k_frame", nblk, 0, n + nblk * HC_BLOCK_SIZE, (uint32_t)grid, 256, kLaneQWords * 4};
  t_last = info;
  return launch_frame(static_cast<const uint8_t *>(src), n, static_cast<uint8_t *>(dst), crc_out, d.dtab, grid,
                      static_cast<hipStream_t>(stream)) == hipSuccess
             ? HC_OK
             : HC_E_HIP;
}

int hc_dev_read_blocks(int device, const void *blocks, uint64_t nblocks, uint32_t block_size, void *payload_out,
                       uint32_t *crc_out, uint32_t *bad_bitmap, int64_t *first_bad, void *stream) {
  if (nblocks == 0) return HC_OK;
  if (!blocks || !payload_out || (bad_bitmap && !first_bad)) return HC_E_ARG;
  uint32_t lg = 0;
  while (lg < 3 && (HC_BLOCK_SIZE << lg) != block_size) lg++;
  if (lg == 3 || (reinterpret_cast<uintptr_t>(blocks) & 15u) != 0) return HC_E_LAYOUT;
  if (unframe_grid(nblocks, lg) > kMaxGridWgs) return HC_E_ARG;  // over 2^32 work-items
  int st = init_device(device);
  if (st != HC_OK) return st;
  DeviceGuard g(device);
  DeviceState &d = g_dev[device];
  hc_launch_info info{"k_unframe", nblocks, 0, nblocks * (2ull * block_size - 4), (uint32_t)unframe_grid(nblocks, lg),
                      256, kLaneQWords * 4};
  t_last = info;
  return launch_unframe(static_cast<const uint8_t *>(blocks), nblocks, lg, static_cast<uint8_t *>(payload_out),
                        crc_out, bad_bitmap, reinterpret_cast<unsigned long long *>(first_bad), d.dtab,
                        static_cast<hipStream_t>(stream)) == hipSuccess
             ? HC_OK
             : HC_E_HIP;
}

int hc_dev_verify_prepare(int device, uint32_t *bad_bitmap, int64_t *first_bad, uint64_t nblocks,
                          void *stream) {
  int st = init_device(device);
  if (st != HC_OK) return st;
  DeviceGuard g(device);
  return launch_verify_prepare(bad_bitmap, reinterpret_cast<unsigned long long *>(first_bad), nblocks,
                               static_cast<hipStream_t>(stream)) == hipSuccess
             ? HC_OK
             : HC_E_HIP;
}

int hc_dev_fill_range(int device, void *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                      uint32_t ulen, uint64_t first_block, uint64_t nblocks, uint64_t seed, void *stream) {
  if (nblocks == 0) return HC_OK;
  if (!base) return HC_E_ARG;
  int st = init_device(device);
  if (st != HC_OK) return st;
  DeviceGuard g(device);
  int grid = (int)std::min<uint64_t>((nblocks + 3) / 4, (uint64_t)g_dev[device].cus * 16);
  return launch_fill(static_cast<uint8_t *>(base), off, len, stride, ulen, nblocks, seed, grid,
                     static_cast<hipStream_t>(stream), first_block) == hipSuccess
             ? HC_OK
             : HC_E_HIP;
}

int hc_dev_fill_blocks(int device, void *base, const uint64_t *off, const uint32_t *len,
                       uint64_t stride, uint32_t ulen, uint64_t nblocks, uint64_t seed, void *stream) {
  return hc_dev_fill_range(device, base, off, len, stride, ulen, 0, nblocks, seed, stream);
}

int hc_host_pipelines(void) { return PipePool::get().live(); }

int hc_stats(hc_stats_t *out) {
  if (!out) return HC_E_ARG;
  auto ld = [](const std::atomic<uint64_t> &a) { return a.load(std::memory_order_relaxed); };
  out->add_crcs_gpu = ld(g_stats.add_crcs_gpu);
  out->add_crcs_host_small = ld(g_stats.add_crcs_host_small);
  out->add_crcs_host_nodev = ld(g_stats.add_crcs_host_nodev);
  out->add_crcs_gpu_fallback = ld(g_stats.add_crcs_gpu_fallback);
  out->last_fallback_error = g_stats.last_fallback_error.load(std::memory_order_relaxed);
  out->read_gpu = ld(g_stats.read_gpu);
  out->read_gpu_fallback = ld(g_stats.read_gpu_fallback);
  out->wal_gpu = ld(g_stats.wal_gpu);
  out->wal_gpu_fallback = ld(g_stats.wal_gpu_fallback);
  out->nodev_host = ld(g_stats.nodev_host);
  return HC_OK;
}

void hc_stats_reset(void) {
  for (auto *a : {&g_stats.add_crcs_gpu, &g_stats.add_crcs_host_small, &g_stats.add_crcs_host_nodev,
                  &g_stats.add_crcs_gpu_fallback, &g_stats.read_gpu, &g_stats.read_gpu_fallback, &g_stats.wal_gpu,
                  &g_stats.wal_gpu_fallback, &g_stats.nodev_host})
    a->store(0);
  g_stats.last_fallback_error.store(0);
}

int hc_last_launch(hc_launch_info *info) {
  if (!info) return HC_E_ARG;
  *info = t_last;
  return HC_OK;
}

int hc_debug_seg_prof(uint64_t *out16) {
  const int dev = t_seg_dev;
  if (dev < 0 || !out16) return HC_E_ARG;
  DeviceGuard g(dev);
  if (hipDeviceSynchronize() != hipSuccess || seg_prof_read(out16) != hipSuccess) return HC_E_HIP;
  return HC_OK;
}

int hc_debug_seg_taken(void) {
  const int dev = t_seg_dev;
  if (dev < 0) return 0;
  DeviceGuard g(dev);
  uint32_t v = 0;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&v, g_dev[dev].seg_last, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return HC_E_HIP;
  return v <= 4 || v == 9 || v == 10 || v == 12 ? (int)v : 0;  // (| 8: the sorted view)
}

int hc_debug_set(const char *name, const char *value) { return hc::knob_set(name, value) ? HC_OK : HC_E_ARG; }

int hc_debug_tables(void *out, size_t cap) {
  if (!out || cap < sizeof(DeviceTables)) return (int)sizeof(DeviceTables);
  std::memcpy(out, &host_tables(), sizeof(DeviceTables));
  return HC_OK;
}

}  // extern "C"
