// kframe3.hip -- round-3 A/B harness for the framing kernels: an LDS-free row
// step for k_frame (AddCRCsToData, row f2) and k_unframe (ReadFromDisk, row f1).
//
// The production kernels keep 144 KiB of replicated byte tables in LDS, so one
// 16-wave workgroup per CU has to fill them before it hashes anything, and the
// kernels run as persistent grids (96-97 % of the persistent
// read+write pattern, which short-lived 4-wave workgroups beat by 5-12 %).
// Here the row step uses no LDS: a 32x32 GF(2) mat-vec M.c is the XOR of six
// 64-entry tables T_j[6-bit chunk j of c], and each table sits in ONE VGPR
// (lane v holds T_j[v]) and is read with ds_bpermute_b32 (the cross-lane
// gather: no LDS allocation, no bank conflicts, no fill).  The tables are
// built per wave from the matrices' 32 columns (scalar loads) in ~6 VALU ops
// per table register, so waves can be short-lived: 4-wave workgroups, K blocks
// per wave, then exit.
//
//   shift(c, 1024)   row step (M)         x^(8*1024)
//   shift(c, 4)      stream combine (S4)   x^32
//   shift(c, 16*2^i) lane placement ladder (T_i, i = 0..5): lane l's value is
//                    shifted by 4 + 16*(63 - l) bytes = S4 * prod T_i^bit_i(63-l)
//
//   ./kframe3 [nblocks=1000000] [rounds=6] [launches=5]
//
// Every variant's output bytes and CRC words are checked against production.
// Not part of the product; build: make -C tools kframe3.
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

namespace xb {

using hc::HC_FRAME_BLOCK;
constexpr int kMats = 8;  // 0: row step, 1: S4, 2..7: T_0..T_5
struct XbCols {
  uint32_t col[kMats][32];
  // the lane placement's per-lane columns (DeviceTables::lane) regrouped for a
  // workgroup-shared LDS copy read by ds_read_b128: lq[q][l][r] = lane[l][4q + r]
  uint32_t lq[8][64][4];
  // Tab5 contents of the row step (0) and shift(., 4) (1): tq[m][j][v] = T_j[v]
  uint32_t tq[2][5][64];
};

inline void build_cols(XbCols &x) {
  hc::Gf2 g;
  const uint64_t n[kMats] = {1024, 4, 16, 32, 64, 128, 256, 512};
  for (int m = 0; m < kMats; m++)
    for (int i = 0; i < 32; i++) x.col[m][i] = g.shift_bytes(1u << i, n[m]);
  hc::DeviceTables h;
  hc::build_device_tables(h);
  for (int q = 0; q < 8; q++)
    for (int l = 0; l < 64; l++)
      for (int r = 0; r < 4; r++) x.lq[q][l][r] = h.lane[l][4 * q + r];
  for (int m = 0; m < 2; m++)
    for (int j = 0; j < 5; j++)
      for (uint32_t v = 0; v < 64; v++) {
        uint32_t e = 0;
        for (int b = 0; b < 6; b++)
          if ((v >> b) & 1u) e ^= x.col[m][6 * j + b];
        x.tq[m][j][v] = e;
      }
}

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// The six chunk tables of one matrix in VGPRs: lane v holds T_j[v] =
// XOR_{b<6, 6j+b<32, bit b of v} col[6j+b].
struct Tab {
  uint32_t t[6];
};
__device__ __forceinline__ Tab make_tab(const uint32_t *__restrict__ col, const uint32_t (&m)[6]) {
  Tab r;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    uint32_t e = 0;
#pragma unroll
    for (int b = 0; b < 6; b++)
      if (6 * j + b < 32) e = __builtin_amdgcn_bitop3_b32(m[b], col[6 * j + b], e, 0x6A);  // (m & c) ^ e
    r.t[j] = e;
  }
  return r;
}

// M.c ^ w through the six tables (kMask: clip each address to bits 7..2)
template <bool kMask>
__device__ __forceinline__ uint32_t apply(const Tab &T, uint32_t c, uint32_t w) {
  uint32_t g[6];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    uint32_t a = j == 0 ? (c << 2) : (c >> (6 * j - 2));
    if (kMask) a &= 0xFCu;
    g[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)a, (int)T.t[j]);
  }
  return x3(x3(g[0], g[1], g[2]), x3(g[3], g[4], g[5]), w);
}

// Hybrid: bits 0..29 of c through five bpermute tables, bits 30..31 on the
// VALU from the matrix's two last columns (wave-uniform), addresses unmasked
// (ds_bpermute reads only address bits 7..2).
struct Tab5 {
  uint32_t t[5];
  uint32_t c30, c31;
};
__device__ __forceinline__ Tab5 make_tab5(const uint32_t *__restrict__ col, const uint32_t (&m)[6]) {
  Tab5 r;
#pragma unroll
  for (int j = 0; j < 5; j++) {
    uint32_t e = 0;
#pragma unroll
    for (int b = 0; b < 6; b++) e = __builtin_amdgcn_bitop3_b32(m[b], col[6 * j + b], e, 0x6A);
    r.t[j] = e;
  }
  r.c30 = col[30];
  r.c31 = col[31];
  return r;
}
__device__ __forceinline__ uint32_t apply5(const Tab5 &T, uint32_t c, uint32_t w) {
  uint32_t g[5];
#pragma unroll
  for (int j = 0; j < 5; j++) g[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j == 0 ? (c << 2) : (c >> (6 * j - 2))), (int)T.t[j]);
  const uint32_t m30 = (uint32_t)((int32_t)(c << 1) >> 31), m31 = (uint32_t)((int32_t)c >> 31);
  uint32_t a = __builtin_amdgcn_bitop3_b32(m30, T.c30, w, 0x6A);
  a = __builtin_amdgcn_bitop3_b32(m31, T.c31, a, 0x6A);
  return x3(x3(g[0], g[1], g[2]), g[3], x3(g[4], a, 0u));
}

// Hybrid framing: row steps and the stream combine through Tab5, the lane
// placement as the production's per-lane 32x32 mat-vec (its columns from the
// constant image, 128 B per lane, loaded once per wave).
template <int K>
__global__ __launch_bounds__(256) void k_frame_xh(const uint8_t *__restrict__ src, uint64_t n,
                                                  uint8_t *__restrict__ dst, uint64_t nblk,
                                                  uint32_t *__restrict__ crc_out, const XbCols *__restrict__ xc,
                                                  const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t kPay = 4092;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * K;
  if (b0 >= nblk) return;
  const uint32_t w0 = tables->w0;
  const bool edge0 = b0 == 0 || b0 == nblk - 1;
  u32x4 v[4];
  auto load4 = [&](uint64_t b) {
    const uint8_t *S = src + b * kPay - 4 + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * hc::kRowBytes));
  };
  if (!edge0) load4(b0);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  uint32_t msk[6];
#pragma unroll
  for (int b = 0; b < 6; b++) msk[b] = 0u - ((lane >> b) & 1u);
  const Tab5 TM = make_tab5(xc->col[0], msk);
  const Tab5 TS = make_tab5(xc->col[1], msk);
  auto finish = [&](const uint32_t (&c)[4]) -> uint32_t {
    const uint32_t d = apply5(TS, apply5(TS, apply5(TS, c[0], c[1]), c[2]), c[3]);
    return hc::wave_xor(hc::matvec32(col, d)) ^ 0xFFFFFFFFu;
  };
  auto row_step = [&](uint32_t c, uint32_t wd) -> uint32_t { return apply5(TM, c, wd); };
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b >= nblk) break;
    uint32_t c[4];
    if (b == 0 || b == nblk - 1) {
      uint4 keep;
      hc::frame_edge_rows(b, src, n, dst, lane, w0, row_step, c, keep);
      const uint32_t crc = finish(c);
      if (lane == 0) {
        keep.x = crc;
        *reinterpret_cast<uint4 *>(dst + b * (uint64_t)HC_FRAME_BLOCK) = keep;
        if (crc_out) crc_out[b] = crc;
      }
      if (k + 1 < K && b + 1 < nblk && b + 1 != nblk - 1) load4(b + 1);
      continue;
    }
    uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      if (r == 0) t.x = lane == 0 ? 0u : t.x;
      __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
    }
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (k + 1 < K && b + 1 < nblk && b + 1 != nblk - 1) load4(b + 1);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) t.x = lane == 0 ? w0 : t.x;
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] = r == 0 ? wd[q] : row_step(c[q], wd[q]);
    }
    const uint32_t crc = finish(c);
    hc::lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crc);
    if (crc_out) hc::lane0_store_u32(crc_out + b, crc);
  }
}

// Interior blocks only (1 .. nblk-2), no edge path (its funnel-shift
// registers raised the kernel to 160+ VGPRs): K blocks per wave, kW waves per
// workgroup; the two edge blocks go to k_frame_edges_xh (one small launch).
template <int K, int kW, int kOcc = 1, int kOrd = 0>
__global__ __attribute__((amdgpu_waves_per_eu(kOcc))) __launch_bounds__(kW * 64) void k_frame_xi(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                      uint64_t nblk, uint32_t *__restrict__ crc_out,
                                                      const XbCols *__restrict__ xc,
                                                      const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t kPay = 4092;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = 1 + ((uint64_t)blockIdx.x * kW + (threadIdx.x >> 6)) * K;  // interior block index + 1
  const uint64_t bend = nblk - 1;
  if (b0 >= bend) return;
  const uint32_t w0 = tables->w0;
  u32x4 v[4];
  auto load4 = [&](uint64_t b) {
    const uint8_t *S = src + b * kPay - 4 + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * hc::kRowBytes));
  };
  load4(b0);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  uint32_t msk[6];
#pragma unroll
  for (int b = 0; b < 6; b++) msk[b] = 0u - ((lane >> b) & 1u);
  const Tab5 TM = make_tab5(xc->col[0], msk);
  const Tab5 TS = make_tab5(xc->col[1], msk);
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b >= bend) break;
    uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
    auto stores = [&](const u32x4 (&src4)[4]) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        u32x4 t = src4[r];
        if (r == 0) t.x = lane == 0 ? 0u : t.x;
        __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
      }
    };
    // kOrd 0: stores, next loads, hash; 1: next loads, stores, hash;
    // 2: next loads, hash, stores (k_unframe's order)
    if (kOrd == 0) stores(v);
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (k + 1 < K && b + 1 < bend) load4(b + 1);
    if (kOrd == 1) stores(cur);
    uint32_t c[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) t.x = lane == 0 ? w0 : t.x;
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] = r == 0 ? wd[q] : apply5(TM, c[q], wd[q]);
    }
    if (kOrd == 2) stores(cur);
    const uint32_t d = apply5(TS, apply5(TS, apply5(TS, c[0], c[1]), c[2]), c[3]);
    const uint32_t crc = hc::wave_xor(hc::matvec32(col, d)) ^ 0xFFFFFFFFu;
    hc::lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crc);
    if (crc_out) hc::lane0_store_u32(crc_out + b, crc);
  }
}

// k_frame_xi with the lane placement's columns shared by the workgroup in LDS
// (8 KiB copied once per workgroup, read with 8 ds_read_b128 per block) instead
// of 128 B loaded per lane: per-wave setup drops to the two Tab5 builds, so
// short-lived waves (K = 1-2 blocks) no longer pay 8 KiB of L2 reads per 8 KiB
// of HBM traffic.
template <int K, int kW, int kOrd = 2, bool kTabLds = false>
__global__ __launch_bounds__(kW * 64) void k_frame_xl(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                      uint64_t nblk, uint32_t *__restrict__ crc_out,
                                                      const XbCols *__restrict__ xc,
                                                      const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t kPay = 4092;
  __shared__ __attribute__((aligned(16))) uint32_t lc[8 * 64 * 4 + (kTabLds ? 2 * 5 * 64 : 0)];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = 1 + ((uint64_t)blockIdx.x * kW + (threadIdx.x >> 6)) * K;
  const uint64_t bend = nblk - 1;
  u32x4 v[4];
  auto load4 = [&](uint64_t b) {
    const uint8_t *S = src + b * kPay - 4 + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * hc::kRowBytes));
  };
  if (b0 < bend) load4(b0);
  {  // lq (8 KiB) and, with kTabLds, tq (2.5 KiB) are contiguous in XbCols
    constexpr int kQ = kTabLds ? 512 + 160 : 512, kT = kW * 64, kPer = (kQ + kT - 1) / kT;
    const uint4 *g = reinterpret_cast<const uint4 *>(&xc->lq[0][0][0]);
    uint4 t[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (threadIdx.x + k * kT < kQ) t[k] = g[threadIdx.x + k * kT];
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (threadIdx.x + k * kT < kQ) reinterpret_cast<uint4 *>(lc)[threadIdx.x + k * kT] = t[k];
  }
  Tab5 TM, TS;
  if (!kTabLds) {
    uint32_t msk[6];
#pragma unroll
    for (int b = 0; b < 6; b++) msk[b] = 0u - ((lane >> b) & 1u);
    TM = make_tab5(xc->col[0], msk);
    TS = make_tab5(xc->col[1], msk);
  } else {
    TM.c30 = xc->col[0][30];
    TM.c31 = xc->col[0][31];
    TS.c30 = xc->col[1][30];
    TS.c31 = xc->col[1][31];
  }
  const uint32_t w0 = tables->w0;
  __syncthreads();
  if (kTabLds) {
#pragma unroll
    for (int j = 0; j < 5; j++) {
      TM.t[j] = lc[2048 + j * 64 + lane];
      TS.t[j] = lc[2048 + 320 + j * 64 + lane];
    }
  }
  if (b0 >= bend) return;
  auto place = [&](uint32_t d) -> uint32_t {
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 c4 = reinterpret_cast<const uint4 *>(lc)[q * 64 + lane];
      const uint32_t cq[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t m = (uint32_t)((int32_t)(d << (31 - (4 * q + r))) >> 31);
        acc = __builtin_amdgcn_bitop3_b32(m, cq[r], acc, 0x6A);  // (m & c) ^ acc
      }
    }
    return acc;
  };
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b >= bend) break;
    uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
    auto stores = [&](const u32x4 (&src4)[4]) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        u32x4 t = src4[r];
        if (r == 0) t.x = lane == 0 ? 0u : t.x;
        __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
      }
    };
    if (kOrd == 0) stores(v);
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (k + 1 < K && b + 1 < bend) load4(b + 1);
    if (kOrd == 1) stores(cur);
    uint32_t c[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) t.x = lane == 0 ? w0 : t.x;
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] = r == 0 ? wd[q] : apply5(TM, c[q], wd[q]);
    }
    if (kOrd == 2) stores(cur);
    const uint32_t d = apply5(TS, apply5(TS, apply5(TS, c[0], c[1]), c[2]), c[3]);
    const uint32_t crc = hc::wave_xor(place(d)) ^ 0xFFFFFFFFu;
    hc::lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crc);
    if (crc_out) hc::lane0_store_u32(crc_out + b, crc);
  }
}

// k_frame_xl (K = 1) with 16-B ALIGNED source loads: each lane loads the
// aligned chunk at its window's start, takes its right neighbour's chunk by a
// whole-wave DPP shift (wave_shl:1, a VALU op, no LDS crossbar) and funnel-
// shifts the pair by the block's misalignment (uniform); lane 63 loads its
// second chunk itself through a buffer range (the other lanes' offsets are out
// of range: no memory access, no branch around the load).  kcopy2 (DESIGN.md
// 4.4a): aligned 4 KiB-per-wave copies 6.0 TB/s, the frame geometry's
// unaligned ones 5.6.
template <int kW>
__global__ __launch_bounds__(kW * 64) void k_frame_xa(const uint8_t *__restrict__ src, uint64_t n,
                                                      uint8_t *__restrict__ dst, uint64_t nblk,
                                                      uint32_t *__restrict__ crc_out, const XbCols *__restrict__ xc,
                                                      const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr uint64_t kPay = 4092;
  __shared__ __attribute__((aligned(16))) uint32_t lc[8 * 64 * 4];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = 1 + (uint64_t)blockIdx.x * kW + (threadIdx.x >> 6);
  const bool mine = b + 1 < nblk;
  const uintptr_t S = (uintptr_t)src + b * kPay - 4;  // source of output byte 0
  const uint32_t m = (uint32_t)(S & 15u), q = m >> 2, rb = m & 3u;
  const uintptr_t Sa = S - m;
  const uintptr_t end = ((uintptr_t)src + n + 15) & ~(uintptr_t)15;  // the range check is per 16-B load
  const uint32_t span = mine ? (uint32_t)(end - Sa < 4112u ? end - Sa : 4112u) : 0u;
  const __amdgpu_buffer_rsrc_t rr = hc::buf_range(reinterpret_cast<const void *>(Sa), span);
  uint4 C[4], X[4];
  if (mine) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Sa + r * hc::kRowBytes + 16u * lane));
      C[r] = make_uint4(t.x, t.y, t.z, t.w);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) X[r] = hc::buf_load16(rr, lane == 63 ? (uint32_t)((r + 1) * hc::kRowBytes) : 0xFFFFFFFFu);
  {
    const uint4 *g = reinterpret_cast<const uint4 *>(&xc->lq[0][0][0]);
    uint4 t[512 / (kW * 64)];
#pragma unroll
    for (int k = 0; k < 512 / (kW * 64); k++) t[k] = g[threadIdx.x + k * kW * 64];
#pragma unroll
    for (int k = 0; k < 512 / (kW * 64); k++) reinterpret_cast<uint4 *>(lc)[threadIdx.x + k * kW * 64] = t[k];
  }
  uint32_t msk[6];
#pragma unroll
  for (int i = 0; i < 6; i++) msk[i] = 0u - ((lane >> i) & 1u);
  const Tab5 TM = make_tab5(xc->col[0], msk);
  const Tab5 TS = make_tab5(xc->col[1], msk);
  const uint32_t w0 = tables->w0;
  __syncthreads();
  if (!mine) return;
  auto shl = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false); };
  u32x4 v[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    uint4 nb = make_uint4(shl(C[r].x), shl(C[r].y), shl(C[r].z), shl(C[r].w));
    if (lane == 63) nb = X[r];
    const uint4 f = hc::funnel16(C[r], nb, q, rb);
    v[r] = u32x4{f.x, f.y, f.z, f.w};
  }
  uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = v[r];
    if (r == 0) t.x = lane == 0 ? 0u : t.x;
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
  }
  uint32_t c[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = v[r];
    if (r == 0) t.x = lane == 0 ? w0 : t.x;
    const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = r == 0 ? wd[k] : apply5(TM, c[k], wd[k]);
  }
  const uint32_t d = apply5(TS, apply5(TS, apply5(TS, c[0], c[1]), c[2]), c[3]);
  uint32_t acc = 0;
#pragma unroll
  for (int qq = 0; qq < 8; qq++) {
    const uint4 c4 = reinterpret_cast<const uint4 *>(lc)[qq * 64 + lane];
    const uint32_t cq[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t mm = (uint32_t)((int32_t)(d << (31 - (4 * qq + r))) >> 31);
      acc = __builtin_amdgcn_bitop3_b32(mm, cq[r], acc, 0x6A);
    }
  }
  const uint32_t crc = hc::wave_xor(acc) ^ 0xFFFFFFFFu;
  hc::lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crc);
  if (crc_out) hc::lane0_store_u32(crc_out + b, crc);
}

// Timing-only twin of k_frame_xa (aligned loads + DPP funnel, XOR fold).
__global__ __launch_bounds__(256) void k_frame_xa_null(const uint8_t *__restrict__ src, uint64_t n,
                                                       uint8_t *__restrict__ dst, uint64_t nblk,
                                                       uint32_t *__restrict__ crc_out) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr uint64_t kPay = 4092;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = 1 + (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b + 1 >= nblk) return;
  const uintptr_t S = (uintptr_t)src + b * kPay - 4;
  const uint32_t m = (uint32_t)(S & 15u), q = m >> 2, rb = m & 3u;
  const uintptr_t Sa = S - m;
  const uintptr_t end = ((uintptr_t)src + n + 15) & ~(uintptr_t)15;
  const __amdgpu_buffer_rsrc_t rr = hc::buf_range(reinterpret_cast<const void *>(Sa), (uint32_t)(end - Sa < 4112u ? end - Sa : 4112u));
  uint4 C[4], X[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Sa + r * hc::kRowBytes + 16u * lane));
    C[r] = make_uint4(t.x, t.y, t.z, t.w);
    X[r] = hc::buf_load16(rr, lane == 63 ? (uint32_t)((r + 1) * hc::kRowBytes) : 0xFFFFFFFFu);
  }
  auto shl = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false); };
  uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
  uint32_t x = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    uint4 nb = make_uint4(shl(C[r].x), shl(C[r].y), shl(C[r].z), shl(C[r].w));
    if (lane == 63) nb = X[r];
    const uint4 f = hc::funnel16(C[r], nb, q, rb);
    __builtin_nontemporal_store(u32x4{f.x, f.y, f.z, f.w}, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
    x ^= f.x ^ f.y ^ f.z ^ f.w;
  }
  x = hc::wave_xor(x);
  if (crc_out) hc::lane0_store_u32(crc_out + b, x);
}

// The production k_unframe (4 KiB blocks) with the lane placement's columns
// shared by the workgroup in LDS (as k_frame_xl) and K blocks per wave.
template <int K, int kW, bool kStoreFirst = false>
__global__ __launch_bounds__(kW * 64) void k_unframe_xl(const uint8_t *__restrict__ blocks, uint64_t nblk,
                                                        uint8_t *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                        uint32_t *__restrict__ bad_bitmap,
                                                        unsigned long long *__restrict__ first_bad,
                                                        const XbCols *__restrict__ xc,
                                                        const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t B = HC_FRAME_BLOCK, Bp = B - 4;
  __shared__ __attribute__((aligned(16))) uint32_t lc[8 * 64 * 4];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = ((uint64_t)blockIdx.x * kW + (threadIdx.x >> 6)) * K;
  const uint64_t p_end = b0 + K < nblk ? b0 + K : nblk;
  uint64_t p = b0;
  const uint32_t w0 = tables->w0;
  u32x4 v[4];
  auto load4 = [&](uint64_t q) {
    const uint8_t *S = blocks + q * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * hc::kRowBytes));
  };
  if (p < p_end) load4(p);
  {
    constexpr int kT = kW * 64, kPer = 512 / kT;
    const uint4 *g = reinterpret_cast<const uint4 *>(&xc->lq[0][0][0]);
    uint4 t[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) t[k] = g[threadIdx.x + k * kT];
#pragma unroll
    for (int k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lc)[threadIdx.x + k * kT] = t[k];
  }
  const hc::XTab TM = hc::make_xtab(tables->tg, lane);
  const hc::XTab TS = hc::make_xtab(tables->s4, lane);
  __syncthreads();
  auto place = [&](uint32_t d) -> uint32_t {
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 c4 = reinterpret_cast<const uint4 *>(lc)[q * 64 + lane];
      const uint32_t cq[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t m = (uint32_t)((int32_t)(d << (31 - (4 * q + r))) >> 31);
        acc = __builtin_amdgcn_bitop3_b32(m, cq[r], acc, 0x6A);
      }
    }
    return acc;
  };
  bool reported = false;
  for (; p < p_end; p++) {
    const uint64_t b = p;
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (K > 1 && p + 1 < p_end) load4(p + 1);
    uint8_t *ob = out + b * Bp + 16u * lane - 4;
    u32x4 sv[4];
    uint8_t *sa[4];
    uint32_t c[4], stored = 0;
    if (kStoreFirst) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const u32x4 t = cur[r];
        if (r == 0) {
          const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);
          const u32x4 first = {t.y, t.z, t.w, nx};
          __builtin_nontemporal_store(lane == 0 ? first : t, reinterpret_cast<u32x4_u *>(ob + (lane == 0 ? 4 : 0)));
        } else {
          __builtin_nontemporal_store(t, reinterpret_cast<u32x4_u *>(ob + r * hc::kRowBytes));
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) {
        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);
        stored = __builtin_amdgcn_readfirstlane(t.x);
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = lane == 0 ? first : t;
        sa[r] = ob + (lane == 0 ? 4 : 0);
        t.x = lane == 0 ? w0 : t.x;
      } else {
        sv[r] = t;
        sa[r] = ob + r * hc::kRowBytes;
      }
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : hc::xapply(TM, c[k], w[k]);
    }
    if (!kStoreFirst) {
#pragma unroll
      for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
    }
    const uint32_t d = hc::xapply(TS, hc::xapply(TS, hc::xapply(TS, c[0], c[1]), c[2]), c[3]);
    const uint32_t crcv = hc::wave_xor(place(d)) ^ 0xFFFFFFFFu;
    if (crc_out) hc::lane0_store_u32(crc_out + b, crcv);
    if (first_bad && crcv != stored) {
      if (bad_bitmap) hc::lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
      if (!reported && b < __hip_atomic_load(first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        hc::lane0_atomic_umin64(first_bad, b);
      reported = true;
    }
  }
}

// The first and the last block (frame_edge_rows: aligned, predicated loads +
// funnel shift), one wave each.
__global__ __launch_bounds__(128) void k_frame_edges_xh(const uint8_t *__restrict__ src, uint64_t n,
                                                        uint8_t *__restrict__ dst, uint64_t nblk,
                                                        uint32_t *__restrict__ crc_out, const XbCols *__restrict__ xc,
                                                        const hc::DeviceTables *__restrict__ tables) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv == 1 && nblk < 2) return;
  const uint64_t b = wv == 0 ? 0 : nblk - 1;
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  uint32_t msk[6];
#pragma unroll
  for (int k = 0; k < 6; k++) msk[k] = 0u - ((lane >> k) & 1u);
  const Tab5 TM = make_tab5(xc->col[0], msk);
  const Tab5 TS = make_tab5(xc->col[1], msk);
  auto row_step = [&](uint32_t c, uint32_t wd) -> uint32_t { return apply5(TM, c, wd); };
  uint32_t c[4];
  uint4 keep;
  hc::frame_edge_rows(b, src, n, dst, lane, tables->w0, row_step, c, keep);
  const uint32_t d = apply5(TS, apply5(TS, apply5(TS, c[0], c[1]), c[2]), c[3]);
  const uint32_t crc = hc::wave_xor(hc::matvec32(col, d)) ^ 0xFFFFFFFFu;
  if (lane == 0) {
    keep.x = crc;
    *reinterpret_cast<uint4 *>(dst + b * (uint64_t)HC_FRAME_BLOCK) = keep;
    if (crc_out) crc_out[b] = crc;
  }
}

// Hybrid ReadFromDisk of 4 KiB blocks (as k_unframe_xb, Tab5 + per-lane placement).
template <int K, int kW = 4, int kOcc = 1>
__global__ __attribute__((amdgpu_waves_per_eu(kOcc))) __launch_bounds__(kW * 64) void k_unframe_xh(const uint8_t *__restrict__ blocks, uint64_t nblk,
                                                    uint8_t *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                    uint32_t *__restrict__ bad_bitmap,
                                                    unsigned long long *__restrict__ first_bad,
                                                    const XbCols *__restrict__ xc,
                                                    const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = ((uint64_t)blockIdx.x * kW + (threadIdx.x >> 6)) * K;
  if (b0 >= nblk) return;
  const uint32_t w0 = tables->w0;
  u32x4 v[4];
  auto load4 = [&](uint64_t b) {
    const uint8_t *S = blocks + b * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * hc::kRowBytes));
  };
  load4(b0);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  uint32_t msk[6];
#pragma unroll
  for (int b = 0; b < 6; b++) msk[b] = 0u - ((lane >> b) & 1u);
  const Tab5 TM = make_tab5(xc->col[0], msk);
  const Tab5 TS = make_tab5(xc->col[1], msk);
  bool reported = false;
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b >= nblk) break;
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (k + 1 < K && b + 1 < nblk) load4(b + 1);
    uint8_t *ob = out + b * (HC_FRAME_BLOCK - 4) + 16u * lane - 4;
    uint32_t c[4], stored = 0;
    u32x4 sv[4];
    uint8_t *sa[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) {
        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);
        stored = __builtin_amdgcn_readfirstlane(t.x);
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = lane == 0 ? first : t;
        sa[r] = ob + (lane == 0 ? 4 : 0);
        t.x = lane == 0 ? w0 : t.x;
      } else {
        sv[r] = t;
        sa[r] = ob + r * hc::kRowBytes;
      }
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] = r == 0 ? wd[q] : apply5(TM, c[q], wd[q]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
    const uint32_t d = apply5(TS, apply5(TS, apply5(TS, c[0], c[1]), c[2]), c[3]);
    const uint32_t crcv = hc::wave_xor(hc::matvec32(col, d)) ^ 0xFFFFFFFFu;
    if (crc_out) hc::lane0_store_u32(crc_out + b, crcv);
    if (first_bad && crcv != stored) {
      if (bad_bitmap) hc::lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
      if (!reported) hc::lane0_atomic_umin64(first_bad, b);
      reported = true;
    }
  }
}

// AddCRCsToData framing (crc_util.go:41-64) of blocks b0 .. b0+K-1 by one wave;
// interior blocks by unaligned 16-B loads, the first and the last block by the
// product's frame_edge_rows (aligned, predicated loads + funnel shift).
template <int K, bool kMask>
__global__ __launch_bounds__(256) void k_frame_xb(const uint8_t *__restrict__ src, uint64_t n,
                                                  uint8_t *__restrict__ dst, uint64_t nblk,
                                                  uint32_t *__restrict__ crc_out, const XbCols *__restrict__ xc,
                                                  const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t kPay = 4092;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t b0 = w * K;
  if (b0 >= nblk) return;
  const uint32_t w0 = tables->w0;
  // the first block's rows go out before the tables are built
  const bool edge0 = b0 == 0 || b0 == nblk - 1;
  u32x4 v[4];
  auto load4 = [&](uint64_t b) {
    const uint8_t *S = src + b * kPay - 4 + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * hc::kRowBytes));
  };
  if (!edge0) load4(b0);
  uint32_t msk[6];
#pragma unroll
  for (int b = 0; b < 6; b++) msk[b] = 0u - ((lane >> b) & 1u);
  const Tab TM = make_tab(xc->col[0], msk);
  const Tab TS = make_tab(xc->col[1], msk);
  Tab TT[6];
#pragma unroll
  for (int i = 0; i < 6; i++) TT[i] = make_tab(xc->col[2 + i], msk);
  const uint32_t place = 63u - lane;
  auto finish = [&](const uint32_t (&c)[4]) -> uint32_t {
    uint32_t d = apply<kMask>(TS, apply<kMask>(TS, apply<kMask>(TS, c[0], c[1]), c[2]), c[3]);
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const uint32_t s = apply<kMask>(TT[i], d, 0u);
      d = ((place >> i) & 1u) ? s : d;
    }
    d = apply<kMask>(TS, d, 0u);
    return hc::wave_xor(d) ^ 0xFFFFFFFFu;
  };
  auto row_step = [&](uint32_t c, uint32_t wd) -> uint32_t { return apply<kMask>(TM, c, wd); };
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b >= nblk) break;
    uint32_t c[4];
    if (b == 0 || b == nblk - 1) {
      uint4 keep;
      hc::frame_edge_rows(b, src, n, dst, lane, w0, row_step, c, keep);
      const uint32_t crc = finish(c);
      if (lane == 0) {
        keep.x = crc;
        *reinterpret_cast<uint4 *>(dst + b * (uint64_t)HC_FRAME_BLOCK) = keep;
        if (crc_out) crc_out[b] = crc;
      }
      if (k + 1 < K && b + 1 < nblk && b + 1 != nblk - 1) load4(b + 1);
      continue;
    }
    uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      if (r == 0) t.x = lane == 0 ? 0u : t.x;
      __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
    }
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (k + 1 < K && b + 1 < nblk && b + 1 != nblk - 1) load4(b + 1);  // next block in flight
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) t.x = lane == 0 ? w0 : t.x;
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] = r == 0 ? wd[q] : row_step(c[q], wd[q]);
    }
    const uint32_t crc = finish(c);
    hc::lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crc);
    if (crc_out) hc::lane0_store_u32(crc_out + b, crc);
  }
}

// Batched ReadFromDisk of 4 KiB blocks (block_manager.go:203-235): verify each
// block and write block[4:] back to back, K blocks per wave, the production
// store order (the block's four rows hashed, then its four payload stores).
template <int K, bool kMask>
__global__ __launch_bounds__(256) void k_unframe_xb(const uint8_t *__restrict__ blocks, uint64_t nblk,
                                                    uint8_t *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                    uint32_t *__restrict__ bad_bitmap,
                                                    unsigned long long *__restrict__ first_bad,
                                                    const XbCols *__restrict__ xc,
                                                    const hc::DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * K;
  if (b0 >= nblk) return;
  const uint32_t w0 = tables->w0;
  u32x4 v[4];
  auto load4 = [&](uint64_t b) {
    const uint8_t *S = blocks + b * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * hc::kRowBytes));
  };
  load4(b0);
  uint32_t msk[6];
#pragma unroll
  for (int b = 0; b < 6; b++) msk[b] = 0u - ((lane >> b) & 1u);
  const Tab TM = make_tab(xc->col[0], msk);
  const Tab TS = make_tab(xc->col[1], msk);
  Tab TT[6];
#pragma unroll
  for (int i = 0; i < 6; i++) TT[i] = make_tab(xc->col[2 + i], msk);
  const uint32_t place = 63u - lane;
  bool reported = false;
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b >= nblk) break;
    u32x4 cur[4] = {v[0], v[1], v[2], v[3]};
    if (k + 1 < K && b + 1 < nblk) load4(b + 1);
    uint8_t *ob = out + b * (HC_FRAME_BLOCK - 4) + 16u * lane - 4;
    uint32_t c[4], stored = 0;
    u32x4 sv[4];
    uint8_t *sa[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = cur[r];
      if (r == 0) {
        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);  // lane+1's x
        stored = __builtin_amdgcn_readfirstlane(t.x);
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = lane == 0 ? first : t;
        sa[r] = ob + (lane == 0 ? 4 : 0);
        t.x = lane == 0 ? w0 : t.x;
      } else {
        sv[r] = t;
        sa[r] = ob + r * hc::kRowBytes;
      }
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] = r == 0 ? wd[q] : apply<kMask>(TM, c[q], wd[q]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
    uint32_t d = apply<kMask>(TS, apply<kMask>(TS, apply<kMask>(TS, c[0], c[1]), c[2]), c[3]);
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const uint32_t s = apply<kMask>(TT[i], d, 0u);
      d = ((place >> i) & 1u) ? s : d;
    }
    d = apply<kMask>(TS, d, 0u);
    const uint32_t crcv = hc::wave_xor(d) ^ 0xFFFFFFFFu;
    if (crc_out) hc::lane0_store_u32(crc_out + b, crcv);
    if (first_bad && crcv != stored) {
      if (bad_bitmap) hc::lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
      if (!reported) hc::lane0_atomic_umin64(first_bad, b);
      reported = true;
    }
  }
}

// Timing-only twin: the same loads, stores and hand-out, the CRC replaced by an
// XOR fold (no tables, no bpermute): the memory pattern's own ceiling.
template <int K>
__global__ __launch_bounds__(256) void k_frame_xb_null(const uint8_t *__restrict__ src, uint64_t n,
                                                       uint8_t *__restrict__ dst, uint64_t nblk,
                                                       uint32_t *__restrict__ crc_out) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t kPay = 4092;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * K;
  for (int k = 0; k < K; k++) {
    const uint64_t b = b0 + k;
    if (b == 0 || b >= nblk - 1) continue;
    const uint8_t *S = src + b * kPay - 4 + 16u * lane;
    uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * hc::kRowBytes));
      __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * hc::kRowBytes));
      x ^= t.x ^ t.y ^ t.z ^ t.w;
    }
    x = hc::wave_xor(x);
    if (crc_out) hc::lane0_store_u32(crc_out + b, x);
  }
}

}  // namespace xb

namespace {
struct Variant {
  std::string name;
  int kind;  // 0 frame, 1 unframe
  bool check;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint64_t npay = N * 4092 - 1000;  // ragged last block, as bench.py --workload frame
  std::printf("device %s, %d CUs; %llu blocks (frame: %llu B payload at an odd address)\n", prop.gcnArchName, cus,
              (unsigned long long)N, (unsigned long long)npay);
  uint8_t *raw, *framed, *framed_ref, *blocks, *pay, *pay_ref;
  uint32_t *crc, *bitmap;
  unsigned long long *fb;
  hc::DeviceTables *dt;
  xb::XbCols *xc;
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
  CK(hipMalloc(&xc, sizeof(xb::XbCols)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
    xb::XbCols x;
    xb::build_cols(x);
    CK(hipMemcpy(xc, &x, sizeof(x), hipMemcpyHostToDevice));
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
  const uint64_t nblk = N;
  std::vector<Variant> vs;
  auto prod_frame = [&](hipStream_t st) { CK(hc::launch_frame(src, npay, framed, crc, dt, cus, st)); };
  auto prod_unframe = [&](hipStream_t st) {
    CK(hc::launch_unframe(blocks, nblk, 0, pay, crc, bitmap, fb, dt, st));
  };
#define XB(K, M)                                                                                                    \
  [&](hipStream_t st) {                                                                                             \
    const uint64_t g_ = (nblk + 4 * (K)-1) / (4 * (K));                                                             \
    hipLaunchKernelGGL((xb::k_frame_xb<K, M>), dim3((unsigned)g_), dim3(256), 0, st, src, npay, framed, nblk, crc, xc, \
                       dt);                                                                                         \
  }
#define XBU(K, M)                                                                                                    \
  [&](hipStream_t st) {                                                                                              \
    const uint64_t g_ = (nblk + 4 * (K)-1) / (4 * (K));                                                              \
    hipLaunchKernelGGL((xb::k_unframe_xb<K, M>), dim3((unsigned)g_), dim3(256), 0, st, blocks, nblk, pay, crc, bitmap, \
                       fb, xc, dt);                                                                                  \
  }
#define XBN(K)                                                                                                   \
  [&](hipStream_t st) {                                                                                          \
    const uint64_t g_ = (nblk + 4 * (K)-1) / (4 * (K));                                                          \
    hipLaunchKernelGGL((xb::k_frame_xb_null<K>), dim3((unsigned)g_), dim3(256), 0, st, src, npay, framed, nblk, crc); \
  }
#define XH(K)                                                                                                   \
  [&](hipStream_t st) {                                                                                         \
    const uint64_t g_ = (nblk + 4 * (K)-1) / (4 * (K));                                                         \
    hipLaunchKernelGGL((xb::k_frame_xh<K>), dim3((unsigned)g_), dim3(256), 0, st, src, npay, framed, nblk, crc, xc, dt); \
  }
#define XHU(K, W, ...)                                                                                            \
  [&](hipStream_t st) {                                                                                              \
    const uint64_t g_ = (nblk + (W) * (K)-1) / ((W) * (K));                                                          \
    hipLaunchKernelGGL((xb::k_unframe_xh<K, W __VA_OPT__(,) __VA_ARGS__>), dim3((unsigned)g_), dim3((W) * 64), 0, st, blocks, nblk, pay, crc,   \
                       bitmap, fb, xc, dt);                                                                          \
  }
#define XI(K, W, ...)                                                                                                \
  [&](hipStream_t st) {                                                                                             \
    hipLaunchKernelGGL(xb::k_frame_edges_xh, dim3(1), dim3(128), 0, st, src, npay, framed, nblk, crc, xc, dt);        \
    const uint64_t g_ = (nblk - 2 + (W) * (K)-1) / ((W) * (K));                                                      \
    hipLaunchKernelGGL((xb::k_frame_xi<K, W __VA_OPT__(,) __VA_ARGS__>), dim3((unsigned)g_), dim3((W) * 64), 0, st, src, framed, nblk, crc, xc, \
                       dt);                                                                                         \
  }
#define XL(K, W, ...)                                                                                                \
  [&](hipStream_t st) {                                                                                             \
    hipLaunchKernelGGL(xb::k_frame_edges_xh, dim3(1), dim3(128), 0, st, src, npay, framed, nblk, crc, xc, dt);        \
    const uint64_t g_ = (nblk - 2 + (W) * (K)-1) / ((W) * (K));                                                      \
    hipLaunchKernelGGL((xb::k_frame_xl<K, W __VA_OPT__(,) __VA_ARGS__>), dim3((unsigned)g_), dim3((W) * 64), 0, st, src, framed, nblk, crc, xc, \
                       dt);                                                                                         \
  }
#define XLU(K, W, ...)                                                                                               \
  [&](hipStream_t st) {                                                                                             \
    const uint64_t g_ = (nblk + (W) * (K)-1) / ((W) * (K));                                                          \
    hipLaunchKernelGGL((xb::k_unframe_xl<K, W __VA_OPT__(,) __VA_ARGS__>), dim3((unsigned)g_), dim3((W) * 64), 0, st, blocks, nblk, pay, crc,   \
                       bitmap, fb, xc, dt);                                                                          \
  }
  const char *only = std::getenv("KF3_SET");  // "xl": the LDS-shared placement study only
#define XA(W)                                                                                                     \
  [&](hipStream_t st) {                                                                                             \
    hipLaunchKernelGGL(xb::k_frame_edges_xh, dim3(1), dim3(128), 0, st, src, npay, framed, nblk, crc, xc, dt);        \
    const uint64_t g_ = (nblk - 2 + (W)-1) / (W);                                                                   \
    hipLaunchKernelGGL((xb::k_frame_xa<W>), dim3((unsigned)g_), dim3((W) * 64), 0, st, src, npay, framed, nblk, crc, \
                       xc, dt);                                                                                     \
  }
  if (only && std::string(only) == "a") {  // aligned source loads for k_frame
    for (int k = 0; k < 2; k++) {
      vs.push_back({"PROD k_frame (unaligned loads)", 0, true, prod_frame, {}});
      vs.push_back({"aligned loads + DPP funnel, W=4", 0, true, XA(4), {}});
      vs.push_back({"NULL np frame K=1 (unaligned)", 0, false, XBN(1), {}});
      vs.push_back({"NULL aligned + DPP funnel", 0, false, [&](hipStream_t st) {
                      const uint64_t g_ = (nblk - 2 + 3) / 4;
                      hipLaunchKernelGGL(xb::k_frame_xa_null, dim3((unsigned)g_), dim3(256), 0, st, src, npay, framed,
                                         nblk, crc);
                    }, {}});
    }
  } else if (only && std::string(only) == "u") {  // unframe geometry only: production against round 3's first build
    for (int k = 0; k < 2; k++) {
      vs.push_back({"PROD k_unframe (K=1, LDS cols)", 1, true, prod_unframe, {}});
      vs.push_back({"per-lane cols unframe K=4 W=4 (r3 first)", 1, true, XHU(4, 4), {}});
    }
  } else if (only && std::string(only) == "xl") {
    vs.push_back({"PROD k_frame (persistent, LDS tables)", 0, true, prod_frame, {}});
    vs.push_back({"hybrid frame interior K=4 W=4 ld,hash,st", 0, true, XI(4, 4, 1, 2), {}});
    vs.push_back({"LDS-cols frame K=1 W=4", 0, true, XL(1, 4), {}});
    vs.push_back({"LDS-cols frame K=1 W=4 st,ld,hash", 0, true, XL(1, 4, 0), {}});
    vs.push_back({"edges only (2 blocks, 1 WG)", 0, false, [&](hipStream_t st) {
                    hipLaunchKernelGGL(xb::k_frame_edges_xh, dim3(1), dim3(128), 0, st, src, npay, framed, nblk, crc, xc, dt);
                  }, {}});
    vs.push_back({"NULL np frame K=1 (memory pattern)", 0, false, XBN(1), {}});
    vs.push_back({"PROD k_frame (again)", 0, true, prod_frame, {}});
    vs.push_back({"PROD k_unframe", 1, true, prod_unframe, {}});
    vs.push_back({"per-lane cols unframe K=4 W=4 (r3 first)", 1, true, XHU(4, 4), {}});
    vs.push_back({"LDS-cols unframe K=1 W=4", 1, true, XLU(1, 4), {}});
    vs.push_back({"LDS-cols unframe K=2 W=4", 1, true, XLU(2, 4), {}});
    vs.push_back({"LDS-cols unframe K=4 W=4", 1, true, XLU(4, 4), {}});
    vs.push_back({"per-lane cols unframe K=4 W=4 (again)", 1, true, XHU(4, 4), {}});
    vs.push_back({"PROD k_unframe (again)", 1, true, prod_unframe, {}});
  } else {
  vs.push_back({"PROD k_frame (persistent, LDS tables)", 0, true, prod_frame, {}});
  vs.push_back({"hybrid frame interior K=4 W=4 st,ld,hash", 0, true, XI(4, 4), {}});
  vs.push_back({"hybrid frame interior K=4 W=4 ld,st,hash", 0, true, XI(4, 4, 1, 1), {}});
  vs.push_back({"hybrid frame interior K=4 W=4 ld,hash,st", 0, true, XI(4, 4, 1, 2), {}});
  vs.push_back({"hybrid frame interior K=8 W=4 ld,hash,st", 0, true, XI(8, 4, 1, 2), {}});
  vs.push_back({"hybrid frame interior K=4 W=8 ld,hash,st", 0, true, XI(4, 8, 1, 2), {}});
  vs.push_back({"hybrid frame interior K=1 W=4 st,ld,hash", 0, true, XI(1, 4), {}});
  vs.push_back({"hybrid frame interior K=2 W=8 ld,hash,st", 0, true, XI(2, 8, 1, 2), {}});
  vs.push_back({"NULL np frame K=1 (memory pattern)", 0, false, XBN(1), {}});
  vs.push_back({"NULL np frame K=4 (memory pattern)", 0, false, XBN(4), {}});
  vs.push_back({"PROD k_unframe (round 3: LDS-free, 4-wave WGs)", 1, true, prod_unframe, {}});
  vs.push_back({"hybrid unframe K=4 W=8", 1, true, XHU(4, 8), {}});
  vs.push_back({"PROD k_frame (again)", 0, true, prod_frame, {}});
  vs.push_back({"PROD k_unframe (round 3, again)", 1, true, prod_unframe, {}});
  }

  // reference outputs: production frame, production unframe (words, bytes, bitmap, first bad)
  std::vector<uint32_t> cref_f(N), cref_u(N), got(N), bm_ref((N + 31) / 32), bm(bm_ref.size());
  unsigned long long fb_ref = 0, fb_got = 0;
  auto prep = [&]() { CK(hc::launch_verify_prepare(bitmap, fb, N, s)); };
  prod_frame(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(framed_ref, framed, N * 4096, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(cref_f.data(), crc, N * 4, hipMemcpyDeviceToHost));
  prep();
  prod_unframe(s);
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
  std::printf("%-42s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double bytes = v.kind ? (double)N * (4096 + 4092) : (double)npay + N * 4096.0;
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-42s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6,
                bytes / med / 1e6 / 80.0, med);
  }
  return bad ? 3 : 0;
}
