// hc_md5.hip — gfx950 kernels for row f4: the Merkle/MD5 integrity check of
// SSTable data (lsm/sstable/sstable.go:2287-2420 CheckIntegrity, leaves
// md5.Sum(record) at :2358; lsm/sstable/merkle_tree/merkle_tree.go:36-81
// parents md5.Sum(left || right)).
//
// MD5 (RFC 1321) chains 64-byte blocks, so one message is one sequential
// chain: the parallelism is across messages.
//   * k_md5_tail (thread per message): writes each message's last one or two
//     padded blocks (data tail, 0x80, zeros, bit length) into a 128-byte slot
//     of a workspace, so the main loop never builds a padded block itself.
//   * k_md5 (lane per message): every lane of a wave pulls messages from the
//     wave's pool as it finishes one (ballot + mbcnt), so the 64 lanes stay
//     busy whatever the message lengths; each iteration a lane hashes one
//     64-byte block: the next full block of its message (four unaligned
//     16-byte loads) or one of its tail blocks from the workspace.  The block
//     function is 64 steps of v_bitop3 (F/G/H/I), v_add3, v_add and v_alignbit
//     (rotate).  Bound: VALU (about 5 ops per byte), not HBM.
//   * k_merkle_level (thread per parent): parent = md5(left || right), one
//     block; an odd level is padded with a zero node (merkle_tree.go:60-66).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hc_kernels.hpp"

namespace hc {

namespace {

__device__ __forceinline__ uint32_t rol(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

// F, G, H, I of RFC 1321 as 3-input truth tables (inputs b = 0xF0, c = 0xCC, d = 0xAA)
template <int kRound>
__device__ __forceinline__ uint32_t fghi(uint32_t b, uint32_t c, uint32_t d) {
  constexpr uint32_t tt = kRound == 0 ? 0xCA : kRound == 1 ? 0xE4 : kRound == 2 ? 0x96 : 0x39;
  return __builtin_amdgcn_bitop3_b32(b, c, d, tt);
}

__device__ __forceinline__ void md5_compress(uint32_t (&st)[4], const uint32_t (&M)[16]) {
  constexpr uint32_t T[64] = {
      0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
      0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
      0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
      0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
      0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
      0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
      0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
      0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
  constexpr int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const int r = i >> 4;
    const int k = r == 0 ? i : r == 1 ? (5 * i + 1) & 15 : r == 2 ? (3 * i + 5) & 15 : (7 * i) & 15;
    uint32_t f;
    if (r == 0)
      f = fghi<0>(b, c, d);
    else if (r == 1)
      f = fghi<1>(b, c, d);
    else if (r == 2)
      f = fghi<2>(b, c, d);
    else
      f = fghi<3>(b, c, d);
    const uint32_t t = d;
    d = c;
    c = b;
    b = b + rol(a + f + M[k] + T[i], S[4 * r + (i & 3)]);
    a = t;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
}

__device__ __forceinline__ void md5_init(uint32_t (&st)[4]) {
  st[0] = 0x67452301u;
  st[1] = 0xefcdab89u;
  st[2] = 0x98badcfeu;
  st[3] = 0x10325476u;
}

__device__ __forceinline__ uint32_t uni_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ---------------------------------------------------------------------------
// Thread per message: the 128-byte tail slot = the message's last len % 64 data
// bytes, 0x80, zeros and the 64-bit little-endian bit length at byte 56 (tail
// < 56 bytes: one block) or 120 (two blocks).  The data bytes come from the
// aligned dwords that hold them (an aligned dword holding a message byte never
// leaves that byte's page), shifted per lane with v_alignbyte.
__global__ __launch_bounds__(256) void k_md5_tail(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
                                                  const uint32_t *__restrict__ lens, uint64_t stride, uint32_t ulen,
                                                  uint64_t n, uint8_t *__restrict__ tails) {
  for (uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = offs ? offs[m] : m * stride;
    const uint32_t l = lens ? lens[m] : ulen;
    const uint32_t r = l & 63u;
    const uintptr_t tp = (uintptr_t)base + o + (l & ~63u);
    const uint32_t sh = (uint32_t)(tp & 3u);
    const uint32_t *A = reinterpret_cast<const uint32_t *>(tp - sh);
    const uint32_t nd = r ? (sh + r + 3) >> 2 : 0u;  // aligned dwords holding the tail bytes (<= 17)
    uint32_t dw[17];
#pragma unroll
    for (int j = 0; j < 17; j++) dw[j] = (uint32_t)j < nd ? __builtin_nontemporal_load(A + j) : 0u;
    uint32_t w[32];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t v = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], sh);
      const int32_t nb = (int32_t)r - 4 * i;  // tail bytes in this word
      v &= nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
      v |= (uint32_t)i == (r >> 2) ? (0x80u << (8 * (r & 3u))) : 0u;
      w[i] = v;
    }
#pragma unroll
    for (int i = 16; i < 32; i++) w[i] = 0;
    const uint64_t bits = (uint64_t)l * 8;
    const bool two = r >= 56;
    w[14] = two ? w[14] : (uint32_t)bits;
    w[15] = two ? w[15] : (uint32_t)(bits >> 32);
    w[30] = two ? (uint32_t)bits : 0u;
    w[31] = two ? (uint32_t)(bits >> 32) : 0u;
    uint4 *dst = reinterpret_cast<uint4 *>(tails + m * 128);
#pragma unroll
    for (int q = 0; q < 8; q++) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
}

// ---------------------------------------------------------------------------
// Lane per message, messages pulled from the wave's pool as lanes free up.
__global__ __launch_bounds__(256) void k_md5(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
                                             const uint32_t *__restrict__ lens, uint64_t stride, uint32_t ulen,
                                             uint64_t n, const uint8_t *__restrict__ tails,
                                             uint8_t *__restrict__ out16) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t wave = uni_u32(threadIdx.x >> 6);
  const uint64_t wpb = blockDim.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + wave, W = (uint64_t)gridDim.x * wpb;
  const uint64_t p1 = n * (gw + 1) / W;
  uint64_t next = n * gw / W;  // wave-uniform pool cursor
  bool act = false;
  uint64_t msg = 0;
  const uint8_t *p = nullptr;   // next full data block
  const uint8_t *tp = nullptr;  // next tail block
  uint32_t nfull = 0, ntail = 0;
  uint32_t st[4] = {0, 0, 0, 0};
  for (;;) {
    const uint64_t need = __ballot(!act);
    if (need) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      const uint64_t idx = next + rank;
      next += (uint64_t)__builtin_popcountll(need);
      if (!act && idx < p1) {
        const uint64_t o = offs ? offs[idx] : idx * stride;
        const uint32_t l = lens ? lens[idx] : ulen;
        msg = idx;
        p = base + o;
        nfull = l >> 6;
        ntail = (l & 63u) < 56 ? 1u : 2u;
        tp = tails + idx * 128;
        md5_init(st);
        act = true;
      }
    }
    if (!__ballot(act)) break;
    if (act) {
      const uint8_t *src = nfull ? p : tp;
      uint32_t M[16];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(src + 16 * q));
        M[4 * q] = v.x;
        M[4 * q + 1] = v.y;
        M[4 * q + 2] = v.z;
        M[4 * q + 3] = v.w;
      }
      md5_compress(st, M);
      if (nfull) {
        p += 64;
        nfull--;
      } else {
        tp += 64;
        if (--ntail == 0) {
          *reinterpret_cast<uint4 *>(out16 + msg * 16) = make_uint4(st[0], st[1], st[2], st[3]);
          act = false;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// One Merkle level: out[i] = md5(in[2i] || in[2i+1]) for i < n_out, with
// in[n_in] read as the zero padding node when n_in is odd; thread n_out writes
// that padding node of `in` (it is serialized with the tree).
__global__ __launch_bounds__(256) void k_merkle_level(uint8_t *__restrict__ in16, uint64_t n_in,
                                                      uint8_t *__restrict__ out16, uint64_t n_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == n_out) {
    if (n_in & 1) *reinterpret_cast<uint4 *>(in16 + n_in * 16) = make_uint4(0, 0, 0, 0);
    return;
  }
  if (i > n_out) return;
  const uint4 L = *reinterpret_cast<const uint4 *>(in16 + 2 * i * 16);
  const uint4 R = 2 * i + 1 < n_in ? *reinterpret_cast<const uint4 *>(in16 + (2 * i + 1) * 16) : make_uint4(0, 0, 0, 0);
  uint32_t M[16] = {L.x, L.y, L.z, L.w, R.x, R.y, R.z, R.w, 0x80u, 0, 0, 0, 0, 0, 256u, 0};
  uint32_t st[4];
  md5_init(st);
  md5_compress(st, M);
  *reinterpret_cast<uint4 *>(out16 + i * 16) = make_uint4(st[0], st[1], st[2], st[3]);
}

__global__ void k_md5_empty(uint8_t *out16) {  // md5.Sum([]byte{}) (merkle_tree.go:37)
  if (threadIdx.x == 0) *reinterpret_cast<uint4 *>(out16) = make_uint4(0xd98c1dd4u, 0x04b2008fu, 0x980980e9u, 0x7e42f8ecu);
}

}  // namespace

hipError_t launch_md5(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t ulen,
                      uint64_t n, uint8_t *tails, uint8_t *out16, int cus, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const int tgrid = (int)((n + 255) / 256 < (uint64_t)cus * 8 ? (n + 255) / 256 : (uint64_t)cus * 8);
  hipLaunchKernelGGL(k_md5_tail, dim3(tgrid), dim3(256), 0, s, base, off, len, stride, ulen, n, tails);
  // 4 waves per workgroup; enough waves that every lane has messages (>= 64 per wave)
  uint64_t waves = (n + 63) / 64;
  const uint64_t maxw = (uint64_t)cus * 32;  // 8 waves per SIMD
  if (waves > maxw) waves = maxw;
  const int grid = (int)((waves + 3) / 4);
  hipLaunchKernelGGL(k_md5, dim3(grid), dim3(256), 0, s, base, off, len, stride, ulen, n, tails, out16);
  return hipGetLastError();
}

hipError_t launch_merkle_levels(uint8_t *levels16, uint64_t n, hipStream_t s) {
  if (n == 0) {
    hipLaunchKernelGGL(k_md5_empty, dim3(1), dim3(64), 0, s, levels16);
    return hipGetLastError();
  }
  uint64_t off = 0, cnt = n;
  while (cnt > 1) {
    const uint64_t padded = cnt + (cnt & 1), nout = padded / 2;
    const int grid = (int)((nout + 1 + 255) / 256);
    hipLaunchKernelGGL(k_merkle_level, dim3(grid), dim3(256), 0, s, levels16 + off * 16, cnt,
                       levels16 + (off + padded) * 16, nout);
    off += padded;
    cnt = nout;
  }
  return hipGetLastError();
}

}  // namespace hc
