// kcopy2.hip — what read+write streams reach on this chip (the ceiling of
// k_frame / k_unframe).  Not part of the product; build: make -C tools kcopy2.
//
//   ./kcopy2 [MiB=4096] [rounds=6] [launches=5]
//
// GB/s = (bytes read + bytes written) / HIP-event launch time, median over
// interleaved rounds; "read" and "write" rows count their one stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

namespace {
typedef float f4 __attribute__((ext_vector_type(4)));

template <int kPol>
__device__ __forceinline__ f4 ld(const f4 *p) {
  if constexpr (kPol == 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int kPol>
__device__ __forceinline__ void st(f4 *p, f4 v) {
  if constexpr (kPol == 1)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// grid-stride float4 copy, U loads in flight per thread before the stores
template <int U, int kLd, int kSt>
__global__ __launch_bounds__(256) void k_copy(const f4 *__restrict__ src, f4 *__restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld<kLd>(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; u++) st<kSt>(dst + i + u * stride, v[u]);
  }
  for (; i < n; i += stride) st<kSt>(dst + i, ld<kLd>(src + i));
}

// block-contiguous: workgroup w copies elements [w*per, (w+1)*per) in tiles of
// 256 threads x U float4
template <int U, int kLd, int kSt>
__global__ __launch_bounds__(256) void k_copy_blk(const f4 *__restrict__ src, f4 *__restrict__ dst, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (size_t t = lo + threadIdx.x; t < hi; t += 256 * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (t + u * 256 < hi) v[u] = ld<kLd>(src + t + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (t + u * 256 < hi) st<kSt>(dst + t + u * 256, v[u]);
  }
}

template <int U, int kLd>
__global__ __launch_bounds__(256) void k_read(const f4 *__restrict__ src, size_t n, float *sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; u++) acc += ld<kLd>(src + i + u * stride);
  }
  if (acc.x == 1234.5f) sink[0] = acc.y;
}

template <int kSt>
__global__ __launch_bounds__(256) void k_write(f4 *__restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const f4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) st<kSt>(dst + i, v);
}

// Persistent copy with the k_crc_grp hand-out: workgroup g owns the chunks of
// 2^kLg consecutive 4 KiB pieces c*G + g; its waves take pieces one at a time
// from an LDS counter (index prefetched one piece ahead).  A wave loads its
// next piece (4 x 1 KiB rows) while it stores the current one.  kLdsKiB pads
// the workgroup's LDS like the product kernels (occupancy).
template <int kWaves, int kLg, int kLdsKiB, int kLd, int kSt>
__global__ __launch_bounds__(kWaves * 64) void k_dyncopy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                         uint64_t npieces, uint32_t *sink) {
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  __shared__ uint32_t ctr;
  if (threadIdx.x == 0) ctr = 2 * kWaves;
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = gridDim.x, g = blockIdx.x;
  auto piece = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> kLg) * G + g) << kLg) | (k & ((1u << kLg) - 1u));
  };
  uint64_t p = piece(wave), pn = piece(kWaves + wave);
  if (p >= npieces) return;
  uint32_t knv = 0;
  if (lane == 0) knv = atomicAdd(&ctr, 1u);
  auto load = [&](uint64_t q, f4 (&v)[4]) {
    const f4 *S = reinterpret_cast<const f4 *>(src + q * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = ld<kLd>(S + r * 64);
  };
  auto store = [&](uint64_t q, const f4 (&v)[4]) {
    f4 *D = reinterpret_cast<f4 *>(dst + q * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) st<kSt>(D + r * 64, v[r]);
  };
  f4 A[4], B[4];
  load(p, A);
  for (;;) {
    bool vn = pn < npieces;
    load(vn ? pn : p, B);
    store(p, A);
    if (!vn) return;
    p = pn;
    pn = piece(__builtin_amdgcn_readfirstlane(knv));
    if (lane == 0) knv = atomicAdd(&ctr, 1u);
    vn = pn < npieces;
    load(vn ? pn : p, A);
    store(p, B);
    if (!vn) return;
    p = pn;
    pn = piece(__builtin_amdgcn_readfirstlane(knv));
    if (lane == 0) knv = atomicAdd(&ctr, 1u);
  }
}

// k_dyncopy with the framing kernels' geometry: piece p reads 4 KiB at
// src + p*sstride + soff and writes it to dst + p*dstride + doff, 16 B per lane
// with unaligned (byte-aligned) vector loads / stores.  frame: sstride 4092,
// soff odd, dstride 4096; unframe: sstride 4096, dstride 4092, doff -4.
template <int kWaves, int kLg, int kLdsKiB>
__global__ __launch_bounds__(kWaves * 64) void k_dyncopy_u(const uint8_t *__restrict__ src, uint64_t sstride,
                                                           int64_t soff, uint8_t *__restrict__ dst, uint64_t dstride,
                                                           int64_t doff, uint64_t npieces, uint32_t *sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  __shared__ uint32_t ctr;
  if (threadIdx.x == 0) ctr = 2 * kWaves;
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = gridDim.x, g = blockIdx.x;
  auto piece = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> kLg) * G + g) << kLg) | (k & ((1u << kLg) - 1u));
  };
  uint64_t p = piece(wave), pn = piece(kWaves + wave);
  if (p >= npieces) return;
  uint32_t knv = 0;
  if (lane == 0) knv = atomicAdd(&ctr, 1u);
  auto load = [&](uint64_t q, u32x4 (&v)[4]) {
    const uint8_t *S = src + q * sstride + soff + 16 * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * 1024));
  };
  auto store = [&](uint64_t q, const u32x4 (&v)[4]) {
    uint8_t *D = dst + q * dstride + doff + 16 * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4_u *>(D + r * 1024));
  };
  u32x4 A[4], B[4];
  load(p, A);
  for (;;) {
    bool vn = pn < npieces;
    load(vn ? pn : p, B);
    store(p, A);
    if (!vn) return;
    p = pn;
    pn = piece(__builtin_amdgcn_readfirstlane(knv));
    if (lane == 0) knv = atomicAdd(&ctr, 1u);
    vn = pn < npieces;
    load(vn ? pn : p, A);
    store(p, B);
    if (!vn) return;
    p = pn;
    pn = piece(__builtin_amdgcn_readfirstlane(knv));
    if (lane == 0) knv = atomicAdd(&ctr, 1u);
  }
}

// Read-only stream with k_crc_grp's geometry and hand-out (16 waves, 144 KiB
// LDS per CU, per-CU chunks of 2^kLg 4 KiB pieces, one piece at a time per
// wave from an LDS counter), kDepth pieces in flight per wave, XOR-folded:
// the memory ceiling of the CRC kernel's pattern at one or two groups in flight.
template <int kDepth, int kLg>
__global__ __launch_bounds__(1024) void k_dynread(const uint8_t *__restrict__ src, uint64_t npieces, uint32_t *sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __shared__ uint32_t lds_pad[144 * 256 + 1];
  __shared__ uint32_t ctr;
  if (threadIdx.x == 0) ctr = kDepth * 16;
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = gridDim.x, g = blockIdx.x;
  auto piece = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> kLg) * G + g) << kLg) | (k & ((1u << kLg) - 1u));
  };
  uint64_t q[kDepth];
#pragma unroll
  for (int d = 0; d < kDepth; d++) q[d] = piece(d * 16 + wave);
  if (q[0] >= npieces) return;
  uint32_t knv = 0;
  if (lane == 0) knv = atomicAdd(&ctr, 1u);
  u32x4 R[kDepth][4];
  auto load = [&](uint64_t p, u32x4 (&v)[4]) {
    const u32x4 *S = reinterpret_cast<const u32x4 *>(src + p * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(S + r * 64);
  };
#pragma unroll
  for (int d = 0; d < kDepth; d++) load(q[d] < npieces ? q[d] : q[0], R[d]);
  // every valid piece is consumed before its slot is refilled; a slot past the
  // end stays past the end (hand-outs increase) and re-reads the last valid piece
  uint32_t acc = 0;
  uint64_t lastv = q[0];
  for (;;) {
    bool alive = false;
#pragma unroll
    for (int d = 0; d < kDepth; d++) {
      const bool v = q[d] < npieces;
      lastv = v ? q[d] : lastv;
#pragma unroll
      for (int r = 0; r < 4; r++) acc ^= R[d][r].x ^ R[d][r].y ^ R[d][r].z ^ R[d][r].w;
      const uint64_t nq = piece(__builtin_amdgcn_readfirstlane(knv));
      if (lane == 0) knv = atomicAdd(&ctr, 1u);
      q[d] = v ? nq : q[d];
      alive = alive || q[d] < npieces;
      load(q[d] < npieces ? q[d] : lastv, R[d]);
    }
    if (!alive) {
      if (acc == 0x12345678u) sink[0] = acc;
      return;
    }
  }
}

// semi-persistent: a workgroup of kWaves waves (optionally holding kLdsKiB of
// LDS, i.e. one workgroup per CU) copies kWaves*kPer consecutive 4 KiB pieces,
// each wave kPer of them one after another (load, store, next), then exits.
// kPer = 1 never waits on a store; larger kPer puts the store acks of piece k
// in front of piece k+1's load wait (in-order vmcnt).
template <int kPer, int kWaves, int kLdsKiB>
__global__ __launch_bounds__(kWaves * 64) void k_npcopy_w(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                          uint64_t npieces, uint32_t *sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = 0; k < kPer; k++) {
    const uint64_t p = ((uint64_t)blockIdx.x * kPer + k) * kWaves + wave;
    if (p >= npieces) return;
    const u32x4 *S = reinterpret_cast<const u32x4 *>(src + p * 4096) + lane;
    u32x4 *D = reinterpret_cast<u32x4 *>(dst + p * 4096) + lane;
    u32x4 v[4];
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(S + r * 64);
#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(v[r], D + r * 64);
  }
}

// Persistent copy split by role: waves 0..7 of a 16-wave workgroup load
// pieces (per-CU chunks of 2^kLg, one piece at a time from an LDS counter,
// the next one in flight) into an LDS ring of kRing 4 KiB slots per wave
// pair; waves 8..15 copy a slot to its destination with global stores and
// never wait on a store (no vmcnt wait in their loop).  LDS: 8*kRing*4 KiB.
template <int kLg, int kRing>
__global__ __launch_bounds__(1024) void k_wscopy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                 uint64_t npieces) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __shared__ u32x4 ring[8][kRing][256];
  __shared__ uint64_t meta[8][kRing];
  __shared__ uint32_t produced[8], consumed[8], ctr;
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t pair = wave & 7;
  if (threadIdx.x < 8) produced[threadIdx.x] = consumed[threadIdx.x] = 0;
  if (threadIdx.x == 0) ctr = 16;
  __syncthreads();
  const uint64_t G = gridDim.x, g = blockIdx.x;
  auto piece = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> kLg) * G + g) << kLg) | (k & ((1u << kLg) - 1u));
  };
  // relaxed workgroup-scope LDS atomics (a volatile generic pointer would be a
  // flat access, which counts on vmcnt and drags every store wait in)
#define LDS_LD(x) __hip_atomic_load(&(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define LDS_ST(x, v) __hip_atomic_store(&(x), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
  if (wave < 8) {
    uint64_t p = piece(wave), pn = piece(8 + wave);
    uint32_t knv = 0;
    if (lane == 0) knv = atomicAdd(&ctr, 1u);
    u32x4 A[4], B[4];
    auto load = [&](uint64_t q, u32x4 (&v)[4]) {
      const u32x4 *S = reinterpret_cast<const u32x4 *>(src + q * 4096) + lane;
#pragma unroll
      for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(S + r * 64);
    };
    if (p < npieces) load(p, A);
    uint32_t t = 0;
    auto put = [&](uint64_t q, const u32x4 (&v)[4], bool data) {
      const uint32_t s = t % kRing;
      while (LDS_LD(consumed[pair]) + kRing < t + 1) __builtin_amdgcn_s_sleep(1);
      if (data) {
#pragma unroll
        for (int r = 0; r < 4; r++) ring[pair][s][r * 64 + lane] = v[r];
      }
      if (lane == 0) LDS_ST(meta[pair][s], q);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) LDS_ST(produced[pair], t + 1);
      t++;
    };
    // X holds piece p (in flight), Y receives the next one; roles alternate
    auto step = [&](u32x4(&X)[4], u32x4(&Y)[4]) -> bool {
      const bool vn = pn < npieces;
      load(vn ? pn : p, Y);
      put(p, X, true);
      p = pn;
      pn = piece(__builtin_amdgcn_readfirstlane(knv));
      if (lane == 0) knv = atomicAdd(&ctr, 1u);
      return vn;
    };
    if (p < npieces)
      while (step(A, B) && step(B, A)) {
      }
    put(~0ull, A, false);
  } else {
    for (uint32_t t = 0;; t++) {
      const uint32_t s = t % kRing;
      while (LDS_LD(produced[pair]) < t + 1) __builtin_amdgcn_s_sleep(1);
      const uint64_t q = LDS_LD(meta[pair][s]);
      if (q == ~0ull) break;
      u32x4 v[4];
#pragma unroll
      for (int r = 0; r < 4; r++) v[r] = ring[pair][s][r * 64 + lane];
      u32x4 *D = reinterpret_cast<u32x4 *>(dst + q * 4096) + lane;
#pragma unroll
      for (int r = 0; r < 4; r++) __builtin_nontemporal_store(v[r], D + r * 64);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) LDS_ST(consumed[pair], t + 1);
    }
  }
#undef LDS_LD
#undef LDS_ST
}

// Persistent copy with a GLOBAL in-order chunk queue, per wave: a wave takes
// chunks of 2^kLg consecutive 4 KiB pieces from one device-wide counter (the
// next chunk's id is requested when the current chunk starts), so all waves of
// the GPU work on neighbouring chunks in request order, as a non-persistent
// grid's workgroups do in dispatch order.  One piece in flight while the
// previous one is stored.  kLdsKiB pads LDS like the product kernels.
template <int kWaves, int kLg, int kLdsKiB>
__global__ __launch_bounds__(kWaves * 64) void k_gqcopy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                        uint64_t npieces, uint32_t *gctr, uint32_t *sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  const uint32_t lane = threadIdx.x & 63;
  constexpr uint32_t C = 1u << kLg;
  uint32_t cur = 0, nxt = 0;
  if (lane == 0) {
    cur = atomicAdd(gctr, 1u);
    nxt = atomicAdd(gctr, 1u);
  }
  cur = __builtin_amdgcn_readfirstlane(cur);
  uint32_t i = 0;
  // next piece of this wave's chunk sequence
  auto take = [&]() -> uint64_t {
    if (i == C) {
      cur = __builtin_amdgcn_readfirstlane(nxt);
      if (lane == 0) nxt = atomicAdd(gctr, 1u);
      i = 0;
    }
    return (uint64_t)cur * C + i++;
  };
  uint64_t p = take();
  if (p >= npieces) return;
  auto load = [&](uint64_t q, u32x4 (&v)[4]) {
    const u32x4 *S = reinterpret_cast<const u32x4 *>(src + q * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(S + r * 64);
  };
  auto store = [&](uint64_t q, const u32x4 (&v)[4]) {
    u32x4 *D = reinterpret_cast<u32x4 *>(dst + q * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(v[r], D + r * 64);
  };
  u32x4 A[4], B[4];
  load(p, A);
  auto step = [&](u32x4(&X)[4], u32x4(&Y)[4]) -> bool {
    const uint64_t pn = take();
    const bool vn = pn < npieces;
    load(vn ? pn : p, Y);
    store(p, X);
    p = pn;
    return vn;
  };
  while (step(A, B) && step(B, A)) {
  }
}

// non-persistent: one workgroup per kPer pieces (k_copy's "one element per
// thread" shape with the framing geometry), no LDS
template <int kPer>
__global__ __launch_bounds__(256) void k_npcopy_u(const uint8_t *__restrict__ src, uint64_t sstride, int64_t soff,
                                                  uint8_t *__restrict__ dst, uint64_t dstride, int64_t doff,
                                                  uint64_t npieces) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = 0; k < kPer; k++) {
    const uint64_t p = (uint64_t)blockIdx.x * 4 * kPer + (uint64_t)k * 4 + wave;
    if (p >= npieces) return;
    const uint8_t *S = src + p * sstride + soff + 16 * lane;
    uint8_t *D = dst + p * dstride + doff + 16 * lane;
    u32x4 v[4];
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * 1024));
#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4_u *>(D + r * 1024));
  }
}

// the same hand-out with static round-robin pieces (piece k of the workgroup
// sequence to wave k % kWaves): isolates the dynamic part
template <int kWaves, int kLg, int kLdsKiB, int kLd, int kSt>
__global__ __launch_bounds__(kWaves * 64) void k_statcopy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                          uint64_t npieces, uint32_t *sink) {
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = gridDim.x, g = blockIdx.x;
  auto piece = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> kLg) * G + g) << kLg) | (k & ((1u << kLg) - 1u));
  };
  uint32_t k = wave;
  uint64_t p = piece(k);
  if (p >= npieces) return;
  f4 A[4];
  for (;;) {
    const f4 *S = reinterpret_cast<const f4 *>(src + p * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) A[r] = ld<kLd>(S + r * 64);
    f4 *D = reinterpret_cast<f4 *>(dst + p * 4096) + lane;
#pragma unroll
    for (int r = 0; r < 4; r++) st<kSt>(D + r * 64, A[r]);
    k += kWaves;
    p = piece(k);
    if (p >= npieces) return;
  }
}

// checks for the role-split / semi-persistent copies: distinct words per
// position, and a device-side compare that counts mismatching 16-B chunks
__global__ void k_iota(uint32_t *a, uint64_t nwords) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 32) ^ 0x5A5A5A5Au;
}
__global__ void k_cmp(const f4 *a, const f4 *b, uint64_t n, unsigned long long *bad) {
  unsigned long long m = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const f4 x = a[i], y = b[i];
    m += __float_as_uint(x.x) != __float_as_uint(y.x) || __float_as_uint(x.y) != __float_as_uint(y.y) ||
         __float_as_uint(x.z) != __float_as_uint(y.z) || __float_as_uint(x.w) != __float_as_uint(y.w);
  }
  if (m) atomicAdd(bad, m);
}

struct Variant {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  const size_t bytes = mib << 20, n = bytes / 16;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("device %s, %d CUs; %zu MiB per stream\n", prop.gcnArchName, cus, mib);
  f4 *a, *b;
  float *sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 256));
  CK(hipMemset(a, 0x5A, bytes));  // non-zero data (DVFS: zeros clock higher)
  CK(hipMemset(b, 0xA5, bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Variant> vs;
  const double rw = 2.0 * bytes;
#define COPY(U, L, S, G) [=](hipStream_t st) { hipLaunchKernelGGL((k_copy<U, L, S>), dim3(G), dim3(256), 0, st, a, b, n); }
#define BLK(U, L, S, G) [=](hipStream_t st) { hipLaunchKernelGGL((k_copy_blk<U, L, S>), dim3(G), dim3(256), 0, st, a, b, n); }
  vs.push_back({"hipMemcpyAsync D2D", rw, [=](hipStream_t st) { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, st)); }, {}});
  vs.push_back({"gs copy U4 pl/pl 8x256/CU", rw, COPY(4, 0, 0, cus * 8), {}});
  vs.push_back({"gs copy U4 nt/nt 8x256/CU", rw, COPY(4, 1, 1, cus * 8), {}});
  vs.push_back({"gs copy U1 pl/pl 8x256/CU", rw, COPY(1, 0, 0, cus * 8), {}});
  vs.push_back({"gs copy U8 pl/pl 8x256/CU", rw, COPY(8, 0, 0, cus * 8), {}});
  vs.push_back({"gs copy U8 nt/nt 8x256/CU", rw, COPY(8, 1, 1, cus * 8), {}});
  vs.push_back({"gs copy U4 pl/pl 4x256/CU", rw, COPY(4, 0, 0, cus * 4), {}});
  vs.push_back({"gs copy U8 pl/pl 2x256/CU", rw, COPY(8, 0, 0, cus * 2), {}});
  vs.push_back({"gs copy U1 pl/pl one thread per f4", rw, COPY(1, 0, 0, (unsigned)(n / 256)), {}});
  vs.push_back({"blk copy U4 pl/pl 8x256/CU", rw, BLK(4, 0, 0, cus * 8), {}});
  vs.push_back({"blk copy U8 nt/nt 8x256/CU", rw, BLK(8, 1, 1, cus * 8), {}});
  vs.push_back({"blk copy U4 pl/nt 8x256/CU", rw, BLK(4, 0, 1, cus * 8), {}});
  const uint64_t np = bytes / 4096;
  const uint8_t *a8 = reinterpret_cast<const uint8_t *>(a);
  uint8_t *b8 = reinterpret_cast<uint8_t *>(b);
#define DYN(W, LG, LDS, L, S, G)                                                                          \
  [=](hipStream_t st) {                                                                                   \
    hipLaunchKernelGGL((k_dyncopy<W, LG, LDS, L, S>), dim3(G), dim3(W * 64), 0, st, a8, b8, np, (uint32_t *)sink); \
  }
#define STAT(W, LG, LDS, L, S, G)                                                                          \
  [=](hipStream_t st) {                                                                                    \
    hipLaunchKernelGGL((k_statcopy<W, LG, LDS, L, S>), dim3(G), dim3(W * 64), 0, st, a8, b8, np, (uint32_t *)sink); \
  }
  vs.push_back({"dyn copy w16 C=32 144KiB LDS nt/nt", rw, DYN(16, 5, 144, 1, 1, cus), {}});
  vs.push_back({"dyn copy w16 C=32 144KiB LDS pl/pl", rw, DYN(16, 5, 144, 0, 0, cus), {}});
  vs.push_back({"dyn copy w16 C=128 144KiB LDS nt/nt", rw, DYN(16, 7, 144, 1, 1, cus), {}});
  vs.push_back({"dyn copy w16 C=8 144KiB LDS nt/nt", rw, DYN(16, 3, 144, 1, 1, cus), {}});
  vs.push_back({"dyn copy w16 C=32 2/CU nt/nt", rw, DYN(16, 5, 1, 1, 1, cus * 2), {}});
  vs.push_back({"dyn copy w8 C=32 4/CU nt/nt", rw, DYN(8, 5, 1, 1, 1, cus * 4), {}});
  vs.push_back({"dyn copy w16 C=32 144KiB nt/pl", rw, DYN(16, 5, 144, 1, 0, cus), {}});
  const uint64_t npu = np - 4;  // leave room for the 4092/4096 stride mismatch
  const double rwu = 2.0 * npu * 4096;
#define DYNU(SS, SO, DS, DO)                                                                                       \
  [=](hipStream_t st) {                                                                                            \
    hipLaunchKernelGGL((k_dyncopy_u<16, 6, 144>), dim3(cus), dim3(1024), 0, st, a8, (uint64_t)(SS), (int64_t)(SO), b8, \
                       (uint64_t)(DS), (int64_t)(DO), npu, (uint32_t *)sink);                                      \
  }
#define NPU(SS, SO, DS, DO)                                                                                        \
  [=](hipStream_t st) {                                                                                            \
    hipLaunchKernelGGL((k_npcopy_u<1>), dim3((unsigned)((npu + 3) / 4)), dim3(256), 0, st, a8, (uint64_t)(SS),     \
                       (int64_t)(SO), b8, (uint64_t)(DS), (int64_t)(DO), npu);                                     \
  }
  const double rd = (double)np * 4096;
#define DYNREAD(D, LG) \
  [=](hipStream_t st) { hipLaunchKernelGGL((k_dynread<D, LG>), dim3(cus), dim3(1024), 0, st, a8, np, (uint32_t *)sink); }
  vs.push_back({"READ dyn 1 piece in flight C=64", rd, DYNREAD(1, 6), {}});
  vs.push_back({"READ dyn 2 pieces in flight C=64", rd, DYNREAD(2, 6), {}});
  vs.push_back({"READ dyn 3 pieces in flight C=64", rd, DYNREAD(3, 6), {}});
  vs.push_back({"READ dyn 1 piece in flight C=128", rd, DYNREAD(1, 7), {}});
  vs.push_back({"READ dyn 2 pieces in flight C=128", rd, DYNREAD(2, 7), {}});
  vs.push_back({"dyn copy_u aligned 4096/4096", rwu, DYNU(4096, 0, 4096, 0), {}});
  vs.push_back({"dyn copy_u FRAME src 4092p+1 -> 4096p", rwu, DYNU(4092, 1, 4096, 0), {}});
  vs.push_back({"dyn copy_u UNFRAME 4096p -> 4092p+12", rwu, DYNU(4096, 0, 4092, 12), {}});
  vs.push_back({"nonpersist copy_u aligned", rwu, NPU(4096, 0, 4096, 0), {}});
  vs.push_back({"nonpersist copy_u FRAME", rwu, NPU(4092, 1, 4096, 0), {}});
  vs.push_back({"nonpersist copy_u UNFRAME", rwu, NPU(4096, 0, 4092, 12), {}});
  vs.push_back({"stat copy w16 C=32 144KiB LDS nt/nt", rw, STAT(16, 5, 144, 1, 1, cus), {}});
  vs.push_back({"stat copy w16 C=1 144KiB LDS nt/nt", rw, STAT(16, 0, 144, 1, 1, cus), {}});
#define NPW(K, W, LDS)                                                                                        \
  [=](hipStream_t st) {                                                                                       \
    hipLaunchKernelGGL((k_npcopy_w<K, W, LDS>), dim3((unsigned)((np + (K) * (W) - 1) / ((K) * (W)))), dim3((W) * 64), 0, \
                       st, a8, b8, np, (uint32_t *)sink);                                                     \
  }
#define WS(LG, R) \
  [=](hipStream_t st) { hipLaunchKernelGGL((k_wscopy<LG, R>), dim3(cus), dim3(1024), 0, st, a8, b8, np); }
  uint32_t *gctr;
  CK(hipMalloc(&gctr, 64));
#define GQ(W, LG, LDS, G)                                                                                     \
  [=](hipStream_t st) {                                                                                       \
    CK(hipMemsetAsync(gctr, 0, 4, st));                                                                       \
    hipLaunchKernelGGL((k_gqcopy<W, LG, LDS>), dim3(G), dim3((W) * 64), 0, st, a8, b8, np, gctr, (uint32_t *)sink); \
  }
  std::vector<std::pair<std::string, std::function<void(hipStream_t)>>> checked = {
      {"gq w16 C=4 144KiB", GQ(16, 2, 144, cus)},  {"gq w16 C=8 144KiB", GQ(16, 3, 144, cus)},
      {"gq w16 C=16 144KiB", GQ(16, 4, 144, cus)}, {"gq w16 C=32 144KiB", GQ(16, 5, 144, cus)},
      {"gq w4 C=8 8/CU", GQ(4, 3, 1, cus * 8)},    {"gq w8 C=8 4/CU", GQ(8, 3, 1, cus * 4)},
      {"gq w8 C=16 4/CU", GQ(8, 4, 1, cus * 4)},   {"gq w16 C=8 2/CU", GQ(16, 3, 1, cus * 2)},
      {"np K=1 w4", NPW(1, 4, 1)},           {"np K=4 w4", NPW(4, 4, 1)},
      {"np K=16 w4", NPW(16, 4, 1)},         {"np K=64 w4", NPW(64, 4, 1)},
      {"np K=1 w16 144KiB", NPW(1, 16, 144)}, {"np K=4 w16 144KiB", NPW(4, 16, 144)},
      {"np K=16 w16 144KiB", NPW(16, 16, 144)}, {"np K=1 w16 no LDS", NPW(1, 16, 1)},
      {"ws C=32 ring 4", WS(5, 4)},          {"ws C=64 ring 4", WS(6, 4)},
      {"ws C=32 ring 2", WS(5, 2)},          {"ws C=32 ring 3", WS(5, 3)},
  };
  for (auto &c : checked) vs.push_back({"copy " + c.first, rw, c.second, {}});
  vs.push_back({"READ only gs U4 pl 8x256/CU", (double)bytes,
                [=](hipStream_t st) { hipLaunchKernelGGL((k_read<4, 0>), dim3(cus * 8), dim3(256), 0, st, a, n, sink); }, {}});
  vs.push_back({"READ only gs U4 nt 8x256/CU", (double)bytes,
                [=](hipStream_t st) { hipLaunchKernelGGL((k_read<4, 1>), dim3(cus * 8), dim3(256), 0, st, a, n, sink); }, {}});
  vs.push_back({"WRITE only gs pl 8x256/CU", (double)bytes,
                [=](hipStream_t st) { hipLaunchKernelGGL((k_write<0>), dim3(cus * 8), dim3(256), 0, st, b, n); }, {}});
  vs.push_back({"WRITE only gs nt 8x256/CU", (double)bytes,
                [=](hipStream_t st) { hipLaunchKernelGGL((k_write<1>), dim3(cus * 8), dim3(256), 0, st, b, n); }, {}});
  int bad = 0;
  {
    unsigned long long *dbad, hbad;
    CK(hipMalloc(&dbad, 8));
    hipLaunchKernelGGL(k_iota, dim3(cus * 8), dim3(256), 0, s, (uint32_t *)a, (uint64_t)(bytes / 4));
    for (auto &c : checked) {
      CK(hipMemsetAsync(b, 0, bytes, s));
      CK(hipMemsetAsync(dbad, 0, 8, s));
      c.second(s);
      hipLaunchKernelGGL(k_cmp, dim3(cus * 8), dim3(256), 0, s, a, b, (uint64_t)(np * 256), dbad);
      CK(hipMemcpyAsync(&hbad, dbad, 8, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      if (hbad) {
        std::printf("MISMATCH copy %s: %llu chunks\n", c.first.c_str(), hbad);
        bad++;
      }
    }
  }
  for (auto &v : vs) v.run(s);
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs)
      for (int l = 0; l < launches; l++) {
        CK(hipEventRecord(e0, s));
        v.run(s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms);
      }
  std::printf("%-40s %10s %10s %8s\n", "variant", "med GB/s", "best GB/s", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-40s %10.1f %10.1f %8.4f\n", v.name.c_str(), v.bytes / med / 1e6, v.bytes / best / 1e6, med);
  }
  return bad ? 3 : 0;
}
