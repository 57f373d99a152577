// kframe4.hip -- round-3 A/B harness for k_frame's neighbour chunk (row f2).
//
// Production k_frame loads each row with aligned 16-B loads and takes lane l's
// second chunk from lane l+1 by DPP; lane 63's second chunk comes from four
// extra buffer loads (one per row) in which every other lane is out of range.
// Those are four more VMEM instructions per wave (8 instead of 4), and the
// timing-only build of that pattern ran 5.47 TB/s against 5.74 for one
// unaligned 16-B load per lane (profiles/r3/framing_lq/r3af_kframe3_aligned.txt).
// Lane 63's chunk of rows 0..2 is lane 0's chunk of the next row, already in
// registers: v_readlane.  Only row 3's (the chunk after the block) needs a load.
//
//   kTail 0  production: four range-predicated buffer loads (lane 63 in range)
//   kTail 1  rows 0..2 by v_readlane of the next row; row 3 by one buffer load
//   kTail 2  rows 0..2 by v_readlane; row 3 by a scalar load of the chunk
//
// Each with its timing-only twin (CRC replaced by an XOR fold), plus the
// unaligned-load copy of round 3.  Outputs of the real variants are checked
// against production byte for byte, CRC words word for word.
//
//   ./kframe4 [nblocks=1000000] [rounds=6] [launches=5]
//
// Not part of the product; build: make -C tools kframe4.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../hunddb_amd/csrc/hc_kernels.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

namespace k4 {
using namespace hc;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 rl0(const u32x4 v) {  // lane 0's chunk, wave-uniform
  return make_uint4(__builtin_amdgcn_readlane(v.x, 0), __builtin_amdgcn_readlane(v.y, 0),
                    __builtin_amdgcn_readlane(v.z, 0), __builtin_amdgcn_readlane(v.w, 0));
}


// XCD-contiguous workgroup order (A/B): workgroup i runs on XCD i % 8; map it to
// logical workgroup (i % 8) * (G / 8) + i / 8 so each XCD's L2 sees one
// contiguous stretch of blocks (the shared boundary lines of neighbouring
// blocks then meet in one L2).  The last G % 8 workgroups keep their index.
__device__ __forceinline__ uint32_t xcd_wg(uint32_t i, uint32_t G) {
  const uint32_t G8 = G & ~7u;
  return i < G8 ? (i & 7u) * (G8 >> 3) + (i >> 3) : i;
}
template <int kTail, bool kNull, bool kGlobal = true, bool kFillFirst = false, bool kXcd = false, bool kMis = false>
__global__ __launch_bounds__(256) void k_frame_t(const uint8_t *__restrict__ src, uint64_t n,
                                                 uint8_t *__restrict__ dst, uint64_t nblk,
                                                 uint32_t *__restrict__ crc_out,
                                                 const DeviceTables *__restrict__ tables) {
  constexpr uint64_t kPay = 4092;
  __shared__ __attribute__((aligned(16))) uint32_t lq[kNull ? 4 : kLaneQWords];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wg = kXcd ? xcd_wg(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t b = 1 + (kMis ? 16ull * (wg >> 2) + 4u * wv + (wg & 3u) : (uint64_t)wg * 4 + wv);  // interior block
  const bool mine = b + 1 < nblk;
  // kGlobal: a wave past the last interior block loads block 1's rows (always
  // interior when this kernel runs) instead of branching around its loads, so
  // the waitcnt pass sees one path and counts the loads exactly
  const uint64_t bl = (kGlobal || kFillFirst) && !mine ? 1 : b;
  const uintptr_t S = (uintptr_t)src + bl * kPay - 4;
  const uint32_t m = (uint32_t)(S & 15u), qs = m >> 2, rs = m & 3u;
  const uintptr_t Sa = S - m;
  // kGlobal: the row address keeps src's provenance (global loads); production
  // computes it as an integer, so hipcc emits flat loads, which also count on
  // lgkmcnt (every scalar-load and LDS wait then waits for the rows too)
  const uint8_t *SaP = kGlobal ? src + (bl * kPay - 4 - m) : reinterpret_cast<const uint8_t *>(Sa);
  const uintptr_t end16 = ((uintptr_t)src + n + 15) & ~(uintptr_t)15;
  const __amdgpu_buffer_rsrc_t r63 =
      buf_range(reinterpret_cast<const void *>(Sa), mine || kGlobal || kFillFirst ? (uint32_t)(end16 - Sa < 4112u ? end16 - Sa : 4112u) : 0u);
  u32x4 C[4];
  uint4 X[4];
  // kFillFirst: the workgroup's LDS copy of the placement columns (L2 hits) is
  // loaded before the rows, so its wait and the barrier need not wait for them
  static_assert(kLaneQWords / 4 / 256 == 2, "two uint4s of columns per thread");
  uint4 lq0, lq1;  // named registers: an array here was promoted to LDS by hipcc
  if constexpr (kFillFirst && !kNull) {
    const uint4 *g = reinterpret_cast<const uint4 *>(&tables->lane_q[0][0][0]);
    lq0 = g[threadIdx.x];
    lq1 = g[threadIdx.x + 256u];
    __builtin_amdgcn_sched_barrier(0);  // keep them ahead of the rows
  }
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  if constexpr (kTail == 3) {  // one unaligned 16-B load per lane: no tail, no funnel
    const uint8_t *SP = kGlobal ? src + (bl * kPay - 4) : reinterpret_cast<const uint8_t *>(S);
#pragma unroll
    for (int r = 0; r < 4; r++)
      C[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(SP + r * kRowBytes + 16u * lane));
  } else if (mine || kGlobal || kFillFirst) {
#pragma unroll
    for (int r = 0; r < 4; r++)
      C[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(SaP + r * kRowBytes + 16u * lane));
  }
  if constexpr (kTail == 0) {
#pragma unroll
    for (int r = 0; r < 4; r++) X[r] = buf_load16(r63, lane == 63 ? (uint32_t)((r + 1) * kRowBytes) : 0xFFFFFFFFu);
  } else if constexpr (kTail == 1) {
    X[3] = buf_load16(r63, lane == 63 ? 4096u : 0xFFFFFFFFu);
  } else if constexpr (kTail == 3) {
  } else {
    // the 16-B chunk after the block's 4096 bytes holds at least one byte of
    // src (b <= nblk-2 and the last block is non-empty), so it lies in src's
    // aligned chunks: a scalar load of it (wave-uniform address) is in bounds
    {
      const uint4 *p = reinterpret_cast<const uint4 *>(SaP + 4096u);
      X[3] = *p;
    }
  }
  if constexpr (kFillFirst) __builtin_amdgcn_sched_barrier(0);  // the rows before the LDS writes
  XTab TM, TS;
  uint32_t w0 = 0;
  if constexpr (!kNull) {
    if constexpr (!kFillFirst) {
      fill_lane_q(lq, tables);
    } else {
      reinterpret_cast<uint4 *>(lq)[threadIdx.x] = lq0;
      reinterpret_cast<uint4 *>(lq)[threadIdx.x + 256u] = lq1;
    }
    TM = make_xtab(tables->tg, lane);
    TS = make_xtab(tables->s4, lane);
    w0 = tables->w0;
    __syncthreads();
  }
  if (!mine) return;
  auto wave_shl1 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false); };
  u32x4 v[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    if constexpr (kTail == 3) {
      v[r] = C[r];
      continue;
    }
    const uint4 a = make_uint4(C[r].x, C[r].y, C[r].z, C[r].w);
    uint4 nb = make_uint4(wave_shl1(a.x), wave_shl1(a.y), wave_shl1(a.z), wave_shl1(a.w));
    if constexpr (kTail == 0) {
      if (lane == 63) nb = X[r];
    } else {
      const uint4 t = r < 3 ? rl0(C[r < 3 ? r + 1 : 3]) : X[3];
      if (lane == 63) nb = t;
    }
    const uint4 f = funnel16(a, nb, qs, rs);
    v[r] = u32x4{f.x, f.y, f.z, f.w};
  }
  uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = v[r];
    if (r == 0) t.x = lane == 0 ? 0u : t.x;
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * kRowBytes));
  }
  uint32_t crcv;
  if constexpr (kNull) {
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) x ^= v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
    crcv = wave_xor(x);
  } else {
    uint32_t c[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      if (r == 0) t.x = lane == 0 ? w0 : t.x;
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : xapply(TM, c[k], w[k]);
    }
    const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
    crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;
  }
  lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crcv);
  if (crc_out) lane0_store_u32(crc_out + b, crcv);
}

// round 3's unaligned-load copy of the frame pattern (one 16-B load per lane per row)
__global__ __launch_bounds__(256) void k_frame_unaligned_null(const uint8_t *__restrict__ src, uint64_t n,
                                                              uint8_t *__restrict__ dst, uint64_t nblk,
                                                              uint32_t *__restrict__ crc_out) {
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = 1 + (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b + 1 >= nblk) return;
  const uint8_t *S = src + b * 4092 - 4 + 16u * lane;
  uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
  uint32_t x = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * kRowBytes));
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * kRowBytes));
    x ^= t.x ^ t.y ^ t.z ^ t.w;
  }
  x = wave_xor(x);
  if (crc_out) lane0_store_u32(crc_out + b, x);
}

// Production k_unframe (4 KiB blocks, one block a wave) with kFillFirst: the
// workgroup's placement columns are loaded before the rows and the first row
// load is unconditional (a wave past the end reads block 0 and exits), so the
// LDS writes and the barrier wait only for the columns (L2 hits), not for
// every wave's rows (production: vmcnt(0) before the LDS writes).
template <bool kFillFirst, bool kXcd = false, bool kEndBar = false, bool kMis = false>
__global__ __launch_bounds__(256) void k_unframe_t(const uint8_t *blocks, uint64_t nblk,  // not restrict: loads stay before the barrier's fence
                                                   uint8_t *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                   uint32_t *__restrict__ bad_bitmap,
                                                   unsigned long long *__restrict__ first_bad,
                                                   const DeviceTables *__restrict__ tables) {
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t Bp = HC_FRAME_BLOCK - 4;
  __shared__ __attribute__((aligned(16))) uint32_t lq[kLaneQWords];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wg = kXcd ? xcd_wg(blockIdx.x, gridDim.x) : blockIdx.x;
  // kMis: workgroup L of a group of four takes blocks 16(L/4) + 4w + L%4, so its
  // four waves' outputs share one misalignment (b mod 4 fixes 4092 b mod 16)
  const uint32_t wvi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t b = kMis ? 16ull * (wg >> 2) + 4u * wvi + (wg & 3u) : (uint64_t)wg * 4 + wvi;
  const bool mine = b < nblk;
  const uint32_t w0 = tables->w0;
  u32x4 v[4];
  uint4 lq0, lq1;
  if constexpr (kFillFirst) {
    const uint4 *g = reinterpret_cast<const uint4 *>(&tables->lane_q[0][0][0]);
    lq0 = g[threadIdx.x];
    lq1 = g[threadIdx.x + 256u];
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t *S = blocks + (mine ? b : 0) * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * kRowBytes));
    __builtin_amdgcn_sched_barrier(0);
    reinterpret_cast<uint4 *>(lq)[threadIdx.x] = lq0;
    reinterpret_cast<uint4 *>(lq)[threadIdx.x + 256u] = lq1;
  } else {
    if (mine) {
      const uint8_t *S = blocks + b * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
      for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * kRowBytes));
    }
    fill_lane_q(lq, tables);
  }
  const XTab TM = make_xtab(tables->tg, lane);
  const XTab TS = make_xtab(tables->s4, lane);
  __syncthreads();
  if (!kEndBar && !mine) return;
  if (kEndBar && !mine) {
    __syncthreads();
    return;
  }
  uint32_t c[4] = {0, 0, 0, 0};
  uint32_t stored = 0;
  uint8_t *ob = out + b * Bp + 16u * lane - 4;
  u32x4 sv[4];
  uint8_t *sa[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = v[r];
    if (r == 0) {
      const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);  // lane+1's x
      stored = __builtin_amdgcn_readfirstlane(t.x);
      const u32x4 first = {t.y, t.z, t.w, nx};
      sv[r] = lane == 0 ? first : t;
      sa[r] = ob + (lane == 0 ? 4 : 0);
      t.x = lane == 0 ? w0 : t.x;
    } else {
      sv[r] = t;
      sa[r] = ob + r * kRowBytes;
    }
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : xapply(TM, c[k], w[k]);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;
  if (crc_out) lane0_store_u32(crc_out + b, crcv);
  if (first_bad && crcv != stored) {
    if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
    if (b < __hip_atomic_load(first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) lane0_atomic_umin64(first_bad, b);
  }
  if constexpr (kEndBar) __syncthreads();  // the workgroup's waves exit together
}

// 4 KiB k_unframe with the payload stores shifted by one word: lane l of row r
// stores block bytes 1024r + 16l + 4 .. +19 at out_b + 1024r + 16l, i.e. its
// own words y, z, w and lane l+1's x (DPP wave_shl:1; lane 63 takes lane 0's
// x of the next row by v_readlane), so no two lanes' stores overlap (the
// production head: lane 0 stores bytes 4..19, overlapping lane 1) and blocks'
// output ranges meet without sharing bytes.  Row 3's lane 63 stores 12 bytes.
__global__ __launch_bounds__(256) void k_unframe_nh(const uint8_t *blocks, uint64_t nblk,
                                                    uint8_t *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                    uint32_t *__restrict__ bad_bitmap,
                                                    unsigned long long *__restrict__ first_bad,
                                                    const DeviceTables *__restrict__ tables) {
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
  typedef u32x3 u32x3_u __attribute__((aligned(1)));
  constexpr uint64_t Bp = HC_FRAME_BLOCK - 4;
  __shared__ __attribute__((aligned(16))) uint32_t lq[kLaneQWords];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool mine = b < nblk;
  const uint32_t w0 = tables->w0;
  u32x4 v[4];
  if (mine) {
    const uint8_t *S = blocks + b * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * kRowBytes));
  }
  fill_lane_q(lq, tables);
  const XTab TM = make_xtab(tables->tg, lane);
  const XTab TS = make_xtab(tables->s4, lane);
  __syncthreads();
  if (!mine) return;
  auto wave_shl1 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false); };
  const uint32_t stored = __builtin_amdgcn_readfirstlane(v[0].x);
  uint8_t *ob = out + b * Bp + 16u * lane;
  u32x4 sv[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    uint32_t nx = wave_shl1(v[r].x);
    if (r < 3) {
      const uint32_t n0 = __builtin_amdgcn_readlane(v[r < 3 ? r + 1 : 3].x, 0);
      nx = lane == 63 ? n0 : nx;
    }
    sv[r] = u32x4{v[r].y, v[r].z, v[r].w, nx};
  }
  uint32_t c[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = v[r];
    if (r == 0) t.x = lane == 0 ? w0 : t.x;
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : xapply(TM, c[k], w[k]);
  }
#pragma unroll
  for (int r = 0; r < 3; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(ob + r * kRowBytes));
  if (lane != 63) {
    __builtin_nontemporal_store(sv[3], reinterpret_cast<u32x4_u *>(ob + 3 * kRowBytes));
  } else {
    const u32x3 t3 = {sv[3].x, sv[3].y, sv[3].z};
    __builtin_nontemporal_store(t3, reinterpret_cast<u32x3_u *>(ob + 3 * kRowBytes));
  }
  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;
  if (crc_out) lane0_store_u32(crc_out + b, crcv);
  if (first_bad && crcv != stored) {
    if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
    if (b < __hip_atomic_load(first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) lane0_atomic_umin64(first_bad, b);
  }
}

// round 3's separate edge launch (the product folds it into k_frame's
// workgroup 0 since late round 3); the harness variants still pair with it
__global__ __launch_bounds__(128) void k_frame_edges_old(const uint8_t *__restrict__ src, uint64_t n,
                                                         uint8_t *__restrict__ dst, uint64_t nblk,
                                                         uint32_t *__restrict__ crc_out,
                                                         const DeviceTables *__restrict__ tables) {
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wv == 1 && nblk < 2) return;
  const uint64_t b = wv == 0 ? 0 : nblk - 1;
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  const XTab TM = make_xtab(tables->tg, lane);
  const XTab TS = make_xtab(tables->s4, lane);
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t { return xapply(TM, c, w); };
  uint32_t c[4];
  uint4 keep;
  frame_edge_rows(b, src, n, dst, lane, tables->w0, row_step, c, keep);
  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
  const uint32_t crcv = wave_xor(matvec32(col, d)) ^ 0xFFFFFFFFu;
  if (lane == 0) {
    keep.x = crcv;
    *reinterpret_cast<uint4 *>(dst + b * (uint64_t)HC_FRAME_BLOCK) = keep;
    if (crc_out) crc_out[b] = crcv;
  }
}
}  // namespace k4

namespace {
struct Variant {
  std::string name;
  int kind;  // 0 frame, 1 unframe
  bool check;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

// KF4_SET: "frame" (k_frame tails), "unframe" (k_unframe column order), "all"
int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  const std::string set = std::getenv("KF4_SET") ? std::getenv("KF4_SET") : "all";
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint64_t npay = N * 4092 - 1000;  // ragged last block, as bench.py --workload frame
  std::printf("device %s, %d CUs; %llu blocks (frame: %llu B payload at an odd address), set %s\n", prop.gcnArchName,
              cus, (unsigned long long)N, (unsigned long long)npay, set.c_str());
  uint8_t *raw, *framed, *framed_ref, *blocks, *pay, *pay_ref;
  uint32_t *crc, *bitmap;
  unsigned long long *fb;
  hc::DeviceTables *dt;
  CK(hipMalloc(&raw, npay + 16));
  CK(hipMalloc(&framed, N * 4096));
  CK(hipMalloc(&framed_ref, N * 4096));
  CK(hipMalloc(&blocks, N * 4096));
  CK(hipMalloc(&pay, N * 4092));
  CK(hipMalloc(&pay_ref, N * 4092));
  CK(hipMalloc(&bitmap, (N + 31) / 32 * 4));
  CK(hipMalloc(&fb, 8));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const uint8_t *src = raw + 1;
  CK(hc::launch_fill(raw, nullptr, nullptr, npay + 16, npay + 16, 1, 0x48756E64, cus * 16, s));
  CK(hc::launch_fill(blocks, nullptr, nullptr, 4096, 4096, N, 0x5EED, cus * 16, s));
  {  // stamp the unframe input, then corrupt every 1000th block
    hc::Batch b{};
    b.base = blocks;
    b.stride = 4096;
    b.ulen = 4096;
    b.nblocks = N;
    b.flags = hc::kFlagStamp;
    b.tables = dt;
    CK(hc::launch_grp(b, cus, s));
    CK(hipStreamSynchronize(s));
    for (uint64_t i = 7; i < N; i += 1000) CK(hipMemsetAsync(blocks + i * 4096 + 100 + (i % 3000), 0x5A, 1, s));
  }
  CK(hipStreamSynchronize(s));
  const uint64_t nblk = (npay + 4091) / 4092;
  const unsigned wgs = (unsigned)((nblk - 2 + 3) / 4);
  auto prod = [&](hipStream_t st) { CK(hc::launch_frame(src, npay, framed, crc, dt, cus, st)); };
  auto prod_u = [&](hipStream_t st) { CK(hc::launch_unframe(blocks, N, 0, pay, crc, bitmap, fb, dt, st)); };
#define KT(T, NUL, G, ...)                                                                                            \
  [&](hipStream_t st) {                                                                                            \
    hipLaunchKernelGGL(k4::k_frame_edges_old, dim3(1), dim3(128), 0, st, src, npay, framed, nblk, crc, dt);             \
    hipLaunchKernelGGL((k4::k_frame_t<T, NUL, G __VA_OPT__(,) __VA_ARGS__>), dim3(wgs), dim3(256), 0, st, src, npay, framed, nblk, crc, dt); \
  }
#define KU(F)                                                                                                  \
  [&](hipStream_t st) {                                                                                        \
    hipLaunchKernelGGL((k4::k_unframe_t<F>), dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, blocks, N, pay, crc, \
                       bitmap, fb, dt);                                                                        \
  }
  std::vector<Variant> vs;
  for (int k = 0; k < 2; k++) {
    if (set == "frame" || set == "all") {
      vs.push_back({"PROD k_frame (4 tail loads)", 0, true, prod, {}});
      vs.push_back({"tail 0 flat (= production, harness copy)", 0, true, KT(0, false, false), {}});
      vs.push_back({"tail 0 global loads", 0, true, KT(0, false, true), {}});
      vs.push_back({"tail 1 global: readlane + 1 buffer load", 0, true, KT(1, false, true), {}});
      vs.push_back({"tail 2 global: readlane + scalar load", 0, true, KT(2, false, true), {}});
      vs.push_back({"tail 2 global, columns loaded first", 0, true, KT(2, false, true, true), {}});
      vs.push_back({"tail 1 flat: readlane + 1 buffer load", 0, true, KT(1, false, false), {}});
      vs.push_back({"tail 1 flat, columns loaded first", 0, true, KT(1, false, false, true), {}});
      vs.push_back({"tail 1 global, columns loaded first", 0, true, KT(1, false, true, true), {}});
      vs.push_back({"NULL tail 0 flat", 0, false, KT(0, true, false), {}});
      vs.push_back({"NULL tail 2 global", 0, false, KT(2, true, true), {}});
      vs.push_back({"NULL unaligned loads", 0, false, [&](hipStream_t st) {
                      hipLaunchKernelGGL(k4::k_frame_unaligned_null, dim3(wgs), dim3(256), 0, st, src, npay, framed,
                                         nblk, crc);
                    }, {}});
    }
    if (set == "ua") {  // k_frame with unaligned row loads in the late-round-3 structure
      vs.push_back({"PROD k_frame", 0, true, prod, {}});
      vs.push_back({"unaligned loads, flat, columns first", 0, true, KT(3, false, false, true), {}});
      vs.push_back({"unaligned loads, global, columns first", 0, true, KT(3, false, true, true), {}});
      vs.push_back({"unaligned loads, global", 0, true, KT(3, false, true), {}});
      vs.push_back({"NULL unaligned loads (round 3 copy)", 0, false, [&](hipStream_t st) {
                      hipLaunchKernelGGL(k4::k_frame_unaligned_null, dim3(wgs), dim3(256), 0, st, src, npay, framed,
                                         nblk, crc);
                    }, {}});
      vs.push_back({"NULL tail 1 flat columns first", 0, false, KT(1, true, false, true), {}});
    }
    if (set == "xcd") {  // XCD-contiguous workgroup order for the short-lived framing kernels
      vs.push_back({"PROD k_frame", 0, true, prod, {}});
      vs.push_back({"frame tail 1 flat FF (2 launches)", 0, true, KT(1, false, false, true), {}});
      vs.push_back({"frame tail 1 flat FF, XCD-contiguous WGs", 0, true, KT(1, false, false, true, true), {}});
      vs.push_back({"frame tail 1 flat FF, XCD, one misalignment per WG", 0, true, [&](hipStream_t st) {
                      hipLaunchKernelGGL(k4::k_frame_edges_old, dim3(1), dim3(128), 0, st, src, npay, framed, nblk, crc, dt);
                      hipLaunchKernelGGL((k4::k_frame_t<1, false, false, true, true, true>),
                                         dim3((unsigned)(4 * ((nblk - 2 + 15) / 16))), dim3(256), 0, st, src, npay,
                                         framed, nblk, crc, dt);
                    }, {}});
      vs.push_back({"NULL frame tail 1 flat FF, XCD-contiguous WGs", 0, false, KT(1, true, false, true, true), {}});
      vs.push_back({"NULL frame tail 1 flat FF", 0, false, KT(1, true, false, true), {}});
      vs.push_back({"PROD k_unframe", 1, true, prod_u, {}});
      vs.push_back({"unframe copy", 1, true, KU(false), {}});
      vs.push_back({"unframe copy, XCD, one misalignment per WG", 1, true, [&](hipStream_t st) {
                      hipLaunchKernelGGL((k4::k_unframe_t<false, true, false, true>), dim3((unsigned)(4 * ((N + 15) / 16))),
                                         dim3(256), 0, st, blocks, N, pay, crc, bitmap, fb, dt);
                    }, {}});
      vs.push_back({"unframe copy, XCD, waves exit together", 1, true, [&](hipStream_t st) {
                      hipLaunchKernelGGL((k4::k_unframe_t<false, true, true>), dim3((unsigned)((N + 3) / 4)), dim3(256), 0,
                                         st, blocks, N, pay, crc, bitmap, fb, dt);
                    }, {}});
      vs.push_back({"unframe copy, XCD-contiguous WGs", 1, true, [&](hipStream_t st) {
                      hipLaunchKernelGGL((k4::k_unframe_t<false, true>), dim3((unsigned)((N + 3) / 4)), dim3(256), 0,
                                         st, blocks, N, pay, crc, bitmap, fb, dt);
                    }, {}});
    }
    if (set == "occf") {  // k_frame at capped occupancy (dynamic LDS padding), edges in their own launch
      vs.push_back({"PROD k_frame (edges in workgroup 0, 68 VGPRs)", 0, true, prod, {}});
      for (uint32_t pad : {0u, 12u, 16u, 24u, 32u}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "tail 1 flat FF + %u KiB LDS pad (%u WGs/CU by LDS)", pad, 160u / (8u + pad));
        vs.push_back({nm, 0, pad == 0, [&, pad](hipStream_t st) {
                        hipLaunchKernelGGL(k4::k_frame_edges_old, dim3(1), dim3(128), 0, st, src, npay, framed, nblk,
                                           crc, dt);
                        hipLaunchKernelGGL((k4::k_frame_t<1, false, false, true>), dim3(wgs), dim3(256), pad << 10, st,
                                           src, npay, framed, nblk, crc, dt);
                      }, {}});
      }
    }
    if (set == "occ") {  // 4 KiB unframe at capped occupancy: dynamic LDS padding limits workgroups per CU
      vs.push_back({"PROD k_unframe", 1, true, prod_u, {}});
      for (uint32_t pad : {0u, 24u, 32u, 40u, 56u}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "unframe copy + %u KiB LDS pad (%u WGs/CU by LDS)", pad, 160u / (8u + pad));
        vs.push_back({nm, 1, pad == 0, [&, pad](hipStream_t st) {
                        hipLaunchKernelGGL(k4::k_unframe_t<false>, dim3((unsigned)((N + 3) / 4)), dim3(256), pad << 10,
                                           st, blocks, N, pay, crc, bitmap, fb, dt);
                      }, {}});
      }
    }
    if (set == "u4") {  // what separates 4 KiB unframe from the 8/16 KiB form: the per-block epilogue?
      vs.push_back({"PROD k_unframe", 1, true, prod_u, {}});
      vs.push_back({"unframe, stores shifted one word (no overlap)", 1, true, [&](hipStream_t st) {
                      hipLaunchKernelGGL(k4::k_unframe_nh, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, blocks,
                                         N, pay, crc, bitmap, fb, dt);
                    }, {}});
      vs.push_back({"PROD k_unframe, no crc_out", 1, false, [&](hipStream_t st) {
                      CK(hc::launch_unframe(blocks, N, 0, pay, nullptr, bitmap, fb, dt, st));
                    }, {}});
      vs.push_back({"PROD k_unframe, no crc_out, no verify", 1, false, [&](hipStream_t st) {
                      CK(hc::launch_unframe(blocks, N, 0, pay, nullptr, nullptr, nullptr, dt, st));
                    }, {}});
      vs.push_back({"PROD k_unframe, crc_out, no verify", 1, false, [&](hipStream_t st) {
                      CK(hc::launch_unframe(blocks, N, 0, pay, crc, nullptr, nullptr, dt, st));
                    }, {}});
    }
    if (set == "unframe" || set == "all") {
      vs.push_back({"PROD k_unframe", 1, true, prod_u, {}});
      vs.push_back({"unframe harness copy (rows, then columns)", 1, true, KU(false), {}});
      vs.push_back({"unframe columns first, unconditional rows", 1, true, KU(true), {}});
    }
  }
  std::vector<uint32_t> cref_f(N), cref_u(N), got(N), bm_ref((N + 31) / 32), bm(bm_ref.size());
  unsigned long long fb_ref = 0, fb_got = 0;
  auto prep = [&]() { CK(hc::launch_verify_prepare(bitmap, fb, N, s)); };
  prod(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(framed_ref, framed, N * 4096, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(cref_f.data(), crc, N * 4, hipMemcpyDeviceToHost));
  prep();
  prod_u(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(pay_ref, pay, N * 4092, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(cref_u.data(), crc, N * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(bm_ref.data(), bitmap, bm_ref.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&fb_ref, fb, 8, hipMemcpyDeviceToHost));
  size_t nbad = 0;
  for (auto w : bm_ref) nbad += __builtin_popcount(w);
  std::printf("reference unframe: %zu bad blocks, first %llu\n", nbad, fb_ref);
  std::vector<uint8_t> h1, h2;
  int bad = 0;
  for (auto &v : vs) {
    if (!v.check) continue;
    const size_t bytes = v.kind ? N * 4092 : N * 4096;
    CK(hipMemsetAsync(crc, 0, N * 4, s));
    CK(hipMemsetAsync(v.kind ? pay : framed, 0x77, bytes, s));
    prep();
    v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), crc, N * 4, hipMemcpyDeviceToHost));
    h1.resize(bytes);
    h2.resize(bytes);
    CK(hipMemcpy(h1.data(), v.kind ? pay : framed, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), v.kind ? pay_ref : framed_ref, bytes, hipMemcpyDeviceToHost));
    size_t wbad = 0, bbad = 0;
    const auto &cref = v.kind ? cref_u : cref_f;
    for (uint64_t i = 0; i < N; i++) wbad += got[i] != cref[i];
    for (size_t i = 0; i < bytes; i++) bbad += h1[i] != h2[i];
    bool vbad = false;
    if (v.kind) {
      CK(hipMemcpy(bm.data(), bitmap, bm.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&fb_got, fb, 8, hipMemcpyDeviceToHost));
      vbad = bm != bm_ref || fb_got != fb_ref;
    }
    if (wbad || bbad || vbad) {
      std::printf("MISMATCH in variant %s: %zu words, %zu bytes, verify %d\n", v.name.c_str(), wbad, bbad, (int)vbad);
      bad++;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs)
      for (int l = 0; l < launches; l++) {
        if (v.kind) prep();
        CK(hipEventRecord(e0, s));
        v.run(s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms);
      }
  std::printf("%-44s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double bytes = v.kind ? (double)N * (4096 + 4092) : (double)npay + N * 4096.0;
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-44s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6,
                bytes / med / 1e6 / 80.0, med);
  }
  return bad ? 3 : 0;
}
