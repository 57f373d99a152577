// hc_md5.hip — gfx950 kernels for row f4: the Merkle/MD5 integrity check of
// SSTable data (lsm/sstable/sstable.go:2287-2420 CheckIntegrity, leaves
// md5.Sum(record) at :2358; lsm/sstable/merkle_tree/merkle_tree.go:36-81
// parents md5.Sum(left || right)).
//
// MD5 (RFC 1321) chains 64-byte blocks, so one message is one sequential
// chain: the parallelism is across messages, one lane per message.
//   * k_md5 (lane per message): lanes take messages as they
//     free up, longest length class first; message bytes reach the lanes in
//     stages of up to 4 blocks, fetched by coalesced 256-byte pieces and
//     swapped through LDS.  The block function is 64 steps of v_bitop3
//     (F/G/H/I), v_add, v_add3, v_alignbit (rotate) and v_add: VALU-bound.
//   * k_merkle_level (thread per parent): parent = md5(left || right), one
//     block; an odd level is padded with a zero node (merkle_tree.go:60-66).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

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
// Lane per message, blocks staged by coalesced loads through LDS.
//
// A lane consumes its message in stages of up to 4 blocks (256 B) and ends it
// with a tail stage: the aligned 16-B chunks holding its last len % 64 bytes,
// padded in the lane's LDS slot into 1-2 blocks (0x80, zeros, bit length; a
// separate tail pass measured no faster).  The 64 stages of a wave are
// fetched by 16 wave-instructions, each covering 4 messages x 256 contiguous
// bytes (16 lanes x 16 B per message): HBM sees >= 128-B pieces, not the 64
// scattered half-lines of a lane-per-message load (1.8 vs 5.5-6.2 TB/s in
// tools/kmd5's probes).  The pieces go to the wave's LDS image (slot m = the
// stage of lane m, odd pitch: conflict-free writes and per-lane ds_read_b128
// at immediate offsets); two stages are in flight while one is compressed
// (kDepth 1 measures within noise of 2: the kernel is VALU-bound at 2 waves
// per SIMD, tools/kmd5).  Pieces past a stage's last valid one
// re-read it: no load leaves a message's full blocks or the aligned chunks
// of its tail.  kStage 3 (3 workgroups per CU) measured slower.
//
// Free lanes take messages from 64-entry metadata windows (lane j holds
// message wbase + j; the next window is prefetched), by ballot rank through
// the pad column of the LDS image.  The wave walks its range once per length
// class, longest first (md5_class).
constexpr int kMd5Waves = 4;        // waves per workgroup; 2 workgroups per CU by LDS
constexpr int kMd5StageBlocks = 4;  // 64-byte blocks per lane per stage
constexpr int kMd5Classes = 4;

// Length class, longest first.  In range order, the lane that draws a 64 KiB
// record last keeps the wave busy alone (+26 % stages for config 5's sizes);
// these four classes come within 1 % of longest-first order.
__device__ __forceinline__ uint32_t md5_class(uint32_t l) {
  return l >= 32768u ? 0u : l >= 8192u ? 1u : l >= 2048u ? 2u : 3u;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

template <bool kOff, bool kLen, int kStage = kMd5StageBlocks, int kDepth = 2, bool kTable = true>
__global__ __launch_bounds__(64 * kMd5Waves) void k_md5(const uint8_t *__restrict__ base,
                                                        const uint64_t *__restrict__ offs,
                                                        const uint32_t *__restrict__ lens, uint64_t stride,
                                                        uint32_t ulen, uint64_t n, uint8_t *__restrict__ out16,
                                                        const uint64_t *__restrict__ bounds) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  // stage pieces are addressed as integers: name the global address space, or
  // they become flat loads, which also count on lgkmcnt (the LDS waits of the
  // compression would wait for the stages in flight: -9 %, tools/kmd5)
  typedef const u32x4 __attribute__((aligned(1), address_space(1))) *gpiece;
  constexpr uint32_t kSlot = 4 * kStage;  // 16-B chunks per stage (<= 16: one 16-lane group per message)
  // slot m (lane m's stage) at m * kPitch chunks: an odd pitch keeps both the
  // loaders' writes and the per-lane ds_read_b128 conflict-free, and every
  // address is a per-lane base plus an immediate offset
  constexpr uint32_t kPitch = kSlot + 1;
  __shared__ u32x4 lds[kMd5Waves][64 * kPitch];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uni_u32(threadIdx.x >> 6);
  u32x4 *L = lds[wave];
  // the hand-off of window entries to free lanes uses the pad column: entry e
  // at chunk e * kPitch + kSlot
  u32x4 *H = L + kSlot;
  const uint64_t gw = (uint64_t)blockIdx.x * kMd5Waves + wave, W = (uint64_t)gridDim.x * kMd5Waves;
  // the wave's messages: equal counts, or equal blocks (bounds: k_md5_bounds)
  const uint64_t p0 = bounds ? bounds[gw] : n * gw / W, p1 = bounds ? bounds[gw + 1] : n * (gw + 1) / W;
  if (p0 >= p1) return;
  // metadata windows: lane j holds message wbase + j; the next window of the
  // walk is prefetched into nw_*
  auto fetch = [&](uint64_t b, uint64_t &o, uint32_t &l) {
    const uint64_t i = b + lane < p1 ? b + lane : p1 - 1;
    // (compile-time layout: a uniform branch around these loads would make the
    // waitcnt pass drain every load in flight at the join)
    if constexpr (kOff)
      o = offs[i];
    else
      o = i * stride;
    if constexpr (kLen)
      l = lens[i];
    else
      l = ulen;
  };
  uint64_t wbase = p0, nwbase = p0, w_off = 0, nw_off = 0;
  uint32_t c = 0, nc = 0, w_len = 0, nw_len = 0;
  auto next_pos = [&]() {
    if (wbase + 64 < p1) {
      nwbase = wbase + 64;
      nc = c;
    } else {
      nwbase = p0;
      nc = c + 1;
    }
    if (nc < (uint32_t)kMd5Classes) fetch(nwbase, nw_off, nw_len);
  };
  fetch(p0, w_off, w_len);
  next_pos();
  uint64_t wmask = __ballot(wbase + lane < p1 && md5_class(w_len) == c);
  bool more = true;  // windows left (wave-uniform)
  bool act = false, fresh = false;
  uint32_t msg = 0;  // message index - p0 (a wave's range is < 2^32 messages)
  uint64_t p = 0;  // address of the message's next full block
  uint32_t nfull = 0, ntail = 0, mlen = 0;
  auto assign = [&]() {
    uint64_t need = __ballot(!act);
    if (!need || !more) return;
    while (need && more) {
      if (!wmask) {
        if (nc >= (uint32_t)kMd5Classes) {
          more = false;
          break;
        }
        wbase = nwbase;
        c = nc;
        w_off = nw_off;
        w_len = nw_len;
        wmask = __ballot(wbase + lane < p1 && md5_class(w_len) == c);
        next_pos();
        continue;
      }
      const uint32_t na = (uint32_t)__builtin_popcountll(need), nw = (uint32_t)__builtin_popcountll(wmask);
      const uint32_t k = na < nw ? na : nw;
      // the first k window entries of the class go to the first k free lanes
      const bool mine = (wmask >> lane) & 1u;
      const uint32_t rj = lane_rank(wmask);
      if (mine && rj < k) H[rj * kPitch] = u32x4{(uint32_t)w_off, (uint32_t)(w_off >> 32), w_len, lane};
      __builtin_amdgcn_wave_barrier();
      const uint32_t r = lane_rank(need);
      if (!act && r < k) {
        const u32x4 h = H[r * kPitch];
        msg = (uint32_t)(wbase - p0) + h.w;
        p = (uint64_t)(uintptr_t)base + (((uint64_t)h.y << 32) | h.x);
        nfull = h.z >> 6;
        ntail = (h.z & 63u) < 56 ? 1u : 2u;
        mlen = h.z;
        act = true;
        fresh = true;
      }
      __builtin_amdgcn_wave_barrier();
      wmask = __ballot(mine && rj >= k);
      need = __ballot(!act);
    }
  };
  // Stages are planned kDepth ahead of the one being compressed: the lane's
  // next blocks of its message (src, nb), or its tail (fin: the digest is
  // complete after it; the lane is free for the next message at once).
  struct Stage {
    uint32_t msg;
    uint32_t nb;  // blocks, 0 = none
    bool first, fin;
    uint32_t tinfo, tlen;  // tail stage: 16-B phase | tail bytes << 4; message length
  };
  // src / cap: the stage's first piece and the offset of its last valid one
  // (pieces past it re-read it)
  auto plan = [&](Stage &t, uint64_t &src, uint32_t &cap) {
    assign();
    t.first = fresh;
    fresh = false;
    t.fin = false;
    t.msg = msg;
    t.tinfo = 0;
    t.tlen = 0;
    if (!act) {
      src = (uint64_t)(uintptr_t)out16;
      cap = 0;
      t.nb = 0;
    } else if (nfull) {
      src = p;
      t.nb = nfull < (uint32_t)kStage ? nfull : (uint32_t)kStage;
      cap = 64u * t.nb - 16u;
      p += 64u * t.nb;
      nfull -= t.nb;
    } else {
      t.nb = ntail;
      t.fin = true;
      act = false;
      // the tail bytes come as the aligned 16-B chunks that hold them (an
      // aligned chunk holding a message byte stays inside that byte's page);
      // compress_stage pads them in place
      const uint32_t r = mlen & 63u, ph = (uint32_t)(p & 15u);
      const uint32_t nck = r ? (ph + r + 15u) >> 4 : 0u;
      src = nck ? (p & ~(uint64_t)15) : (uint64_t)(uintptr_t)out16;
      cap = nck ? 16u * (nck - 1u) : 0u;
      t.tinfo = ph | (r << 4);
      t.tlen = mlen;
    }
  };
  // 16 wave-instructions per stage; each covers 4 messages x kSlot chunks
  // (lanes 16r + j, j < kSlot; with kSlot < 16 the other lanes re-read a piece)
  const uint32_t pj = 16u * (lane & 15u);  // this lane's piece offset in every stage
  auto issue = [&](u32x4(&R)[16], uint64_t src, uint32_t cap) {
    if constexpr (kTable) {
      // every lane posts {src, cap} in the pad column of its slot (the
      // hand-off is done by now); a loader reads the 16 entries it serves,
      // broadcast within its 16-lane group: 1 + 16 LDS instructions instead
      // of 48 ds_bpermute
      __builtin_amdgcn_wave_barrier();
      H[lane * kPitch] = u32x4{(uint32_t)src, (uint32_t)(src >> 32), cap, 0u};
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t q = 0; q < 16; q++) {
        const u32x4 e = H[(4u * q + (lane >> 4)) * kPitch];
        const uint64_t t = ((uint64_t)e.y << 32) | e.x;
        R[q] = *(gpiece)(t + (pj < e.z ? pj : e.z));
      }
      __builtin_amdgcn_wave_barrier();
    } else {
#pragma unroll
      for (uint32_t q = 0; q < 16; q++) {
        const uint32_t m = 4u * q + (lane >> 4);
        const uint64_t t = ((uint64_t)shfl32((uint32_t)(src >> 32), m) << 32) | shfl32((uint32_t)src, m);
        const uint32_t mc = shfl32(cap, m);
        R[q] = *(gpiece)(t + (pj < mc ? pj : mc));
      }
    }
  };
  uint32_t st[4] = {0, 0, 0, 0};
  auto compress_stage = [&](const Stage &t) {
    if (t.first) md5_init(st);
    {
      if (t.fin) {
        // the padded tail blocks, built in the lane's own slot: the last
        // len % 64 bytes (funnel-shifted out of the aligned chunks), 0x80,
        // zeros, the bit length at byte 56 (or 120: a second block)
        const uint32_t ph = t.tinfo & 15u, r = t.tinfo >> 4, sh = ph & 3u;
        const uint32_t *Dw = reinterpret_cast<const uint32_t *>(L + lane * kPitch) + (ph >> 2);
        uint32_t w[16];
        uint32_t lo = Dw[0];
#pragma unroll
        for (int k = 0; k < 16; k++) {
          const uint32_t hi = Dw[k + 1];
          uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);
          lo = hi;
          const int32_t nbk = (int32_t)r - 4 * k;  // tail bytes in this word
          v &= nbk >= 4 ? 0xFFFFFFFFu : (nbk <= 0 ? 0u : (1u << (8 * nbk)) - 1u);
          v |= (uint32_t)k == (r >> 2) ? (0x80u << (8 * (r & 3u))) : 0u;
          w[k] = v;
        }
        const uint64_t bits = (uint64_t)t.tlen * 8;
        const bool two = r >= 56;
        if (!two) {
          w[14] = (uint32_t)bits;
          w[15] = (uint32_t)(bits >> 32);
        }
        u32x4 *S = L + lane * kPitch;
#pragma unroll
        for (int k = 0; k < 4; k++) S[k] = u32x4{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
        if (two) {
          S[4] = u32x4{0u, 0u, 0u, 0u};
          S[5] = u32x4{0u, 0u, 0u, 0u};
          S[6] = u32x4{0u, 0u, 0u, 0u};
          S[7] = u32x4{0u, 0u, (uint32_t)bits, (uint32_t)(bits >> 32)};
        }
      }
    }
    for (uint32_t b = 0; b < (uint32_t)kStage; b++) {
      if (b < t.nb) {
        uint32_t M[16];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          const u32x4 v = L[lane * kPitch + 4u * b + q];
          M[4 * q] = v.x;
          M[4 * q + 1] = v.y;
          M[4 * q + 2] = v.z;
          M[4 * q + 3] = v.w;
        }
        md5_compress(st, M);
      }
    }
    if (t.fin) *reinterpret_cast<uint4 *>(out16 + (p0 + t.msg) * 16) = make_uint4(st[0], st[1], st[2], st[3]);
  };
  u32x4 R[kDepth][16];
  Stage T[kDepth];
#pragma unroll
  for (int d = 0; d < kDepth; d++) {
    uint64_t src;
    uint32_t cap;
    plan(T[d], src, cap);
    issue(R[d], src, cap);
  }
  // one step on register set d (a template argument, so R[d] stays in registers)
  auto step = [&](auto dc) -> bool {
    constexpr int d = decltype(dc)::value;
    // the oldest stage empty everywhere: so are the later ones
    if (!__ballot(T[d].nb != 0)) return false;
    // pieces -> LDS: chunk j of slot m at m * kPitch + j
#pragma unroll
    for (uint32_t q = 0; q < 16; q++)
      if ((lane & 15u) < kSlot) L[(4u * q + (lane >> 4)) * kPitch + (lane & 15u)] = R[d][q];
    __builtin_amdgcn_wave_barrier();
    const Stage cur = T[d];
    uint64_t src;
    uint32_t cap;
    plan(T[d], src, cap);
    issue(R[d], src, cap);  // in flight while the older stages are compressed
    compress_stage(cur);
    __builtin_amdgcn_wave_barrier();
    return true;
  };
  static_assert(kDepth == 1 || kDepth == 2, "one register set, or two used alternately");
  if constexpr (kDepth == 2) {
    while (step(std::integral_constant<int, 0>{}) && step(std::integral_constant<int, 1>{})) {
    }
  } else {
    while (step(std::integral_constant<int, 0>{})) {
    }
  }
}

// ---------------------------------------------------------------------------
// Ranges of equal work for k_md5's waves (variable lengths).  Equal message
// counts left the heaviest of 2048 waves 16.8 % above the mean on 2M
// log-uniform records (64 B - 64 KiB: a wave's ~1000 records sum to 9.5 MB
// +- 5 %), and the kernel waits for it.  The work of a message is its
// compressions, md5_blocks(len).  Three small launches: chunk sums, their
// scan and each wave's chunk, the split inside that chunk.
constexpr uint32_t kMd5Chunk = 2048;    // messages per weight chunk
constexpr uint32_t kMd5MaxWaves = 8192; // k_md5's largest grid (x kMd5Waves)
constexpr uint32_t kMd5MaxChunks = 16384;  // k_md5_split's prefix in LDS (128 KiB): up to 32M messages

__device__ __forceinline__ uint32_t md5_blocks(uint32_t l) { return (l >> 6) + ((l & 63u) < 56u ? 1u : 2u); }

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, d);
  return v;
}

// csum[c] = the compressions of chunk c (one workgroup a chunk)
__global__ __launch_bounds__(256) void k_md5_wsum(const uint32_t *__restrict__ lens, uint64_t n,
                                                  unsigned long long *__restrict__ csum) {
  __shared__ unsigned long long part[4];
  const uint64_t lo = (uint64_t)blockIdx.x * kMd5Chunk, hi = lo + kMd5Chunk < n ? lo + kMd5Chunk : n;
  uint64_t v = 0;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += 256) v += md5_blocks(lens[i]);
  v = wave_sum_u64(v);
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) csum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// One workgroup: csum -> exclusive prefix (in place, csum[nch] = total), then
// for every wave g in 1 .. W-1 its target T_g = total * g / W and the chunk
// holding it: gch[g] = the last chunk c with csum[c] <= T_g, gt[g] = T_g.
__global__ __launch_bounds__(1024) void k_md5_split(unsigned long long *__restrict__ csum, uint64_t nch,
                                                    uint32_t W, unsigned long long *__restrict__ gch,
                                                    unsigned long long *__restrict__ gt) {
  __shared__ unsigned long long wsum[16];
  __shared__ unsigned long long carry;
  __shared__ unsigned long long pre[kMd5MaxChunks];  // the search reads the prefix here, not
                                                     // through the vector L1 it was read into
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nch; base += 1024) {
    const uint64_t i = base + t;
    const uint64_t v = i < nch ? csum[i] : 0;
    uint64_t x = v;  // inclusive scan within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, d);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t off = carry;
    for (uint32_t k = 0; k < wv; k++) off += wsum[k];
    if (i < nch) csum[i] = pre[i] = off + x - v;  // exclusive
    __syncthreads();
    if (t == 1023) carry = off + x;
    __syncthreads();
  }
  const uint64_t total = carry;
  if (t == 0) csum[nch] = total;
  for (uint32_t g = 1 + t; g < W; g += 1024) {
    const uint64_t T = (total / W) * g + ((total % W) * g) / W;
    uint64_t lo = 0, hi = nch;  // the last c < nch with csum[c] <= T (csum[0] = 0)
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (pre[mid] <= T)
        lo = mid;
      else
        hi = mid;
    }
    gch[g] = lo;
    gt[g] = T;
  }
}

// One wave per split g: bounds[g] = the first message whose exclusive prefix
// of compressions is >= T_g (in chunk gch[g], or the next chunk's first);
// bounds[0] = 0, bounds[W] = n.  Monotone in g, so the ranges tile [0, n).
__global__ __launch_bounds__(256) void k_md5_bounds(const uint32_t *__restrict__ lens, uint64_t n, uint32_t W,
                                                    const unsigned long long *__restrict__ csum,
                                                    const unsigned long long *__restrict__ gch,
                                                    const unsigned long long *__restrict__ gt,
                                                    uint64_t *__restrict__ bounds) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (g > W) return;  // whole waves
  if (g == 0 || g == W) {
    if (lane == 0) bounds[g] = g ? n : 0;
    return;
  }
  constexpr uint32_t kPer = kMd5Chunk / 64;
  const uint64_t c = gch[g], T = gt[g], lo = c * kMd5Chunk;
  uint32_t w[kPer];
  uint64_t ls = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint64_t i = lo + lane * kPer + k;
    w[k] = i < n ? md5_blocks(lens[i]) : 0u;
    ls += w[k];
  }
  uint64_t x = ls;  // inclusive scan of the lane sums
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  // exclusive prefix of this lane's first message; the message of the lane's
  // range where the running prefix first reaches T
  uint64_t run = csum[c] + x - ls, idx = ~0ull;
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint64_t i = lo + lane * kPer + k;
    if (idx == ~0ull && run >= T && i < n) idx = i;
    run += w[k];
  }
  // the lowest lane's hit; none: the next chunk's first message
  uint64_t best = idx;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = (uint64_t)__shfl_xor((unsigned long long)best, d);
    best = o < best ? o : best;
  }
  if (lane == 0) {
    const uint64_t nx = lo + kMd5Chunk < n ? lo + kMd5Chunk : n;
    bounds[g] = best != ~0ull ? best : nx;
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

// messages from which k_md5's waves get ranges of equal work (off/len batches)
constexpr uint64_t kMd5BalanceMin = 16384;

// workspace: the chunk sums and their prefix (nch + 1), each wave's chunk and
// target (kMd5MaxWaves + 1 each), the ranges (kMd5MaxWaves + 1); u64 words
uint64_t md5_workspace_bytes(uint64_t n) {
  const uint64_t nch = (n + kMd5Chunk - 1) / kMd5Chunk;
  if (n < kMd5BalanceMin || nch > kMd5MaxChunks) return 0;
  return 8 * ((nch + 1) + 3 * ((uint64_t)kMd5MaxWaves + 1));
}

hipError_t launch_md5(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t ulen,
                      uint64_t n, uint8_t *workspace, uint8_t *out16, int cus, hipStream_t s) {
  if (n == 0) return hipSuccess;
  // 2 workgroups (8 waves) per CU fit the LDS; a smaller batch gets 4 messages
  // per lane per wave range (256 per wave): with heavy-tailed sizes, fewer and
  // longer ranges balance better than more waves (200k log-uniform records:
  // 1991 GB/s at 196 workgroups against 1284 at 512, profiles/r1/md5/dyn/)
  uint64_t grid = (n + 256 * kMd5Waves - 1) / (256 * kMd5Waves);
  if (grid > (uint64_t)cus * 2) grid = (uint64_t)cus * 2;
  const uint32_t W = (uint32_t)grid * kMd5Waves;
  const uint64_t *bounds = nullptr;
  const uint64_t nch = (n + kMd5Chunk - 1) / kMd5Chunk;
  if (len && workspace && n >= kMd5BalanceMin && W <= kMd5MaxWaves && nch <= kMd5MaxChunks) {  // equal work
    auto *csum = reinterpret_cast<unsigned long long *>(workspace);
    unsigned long long *gch = csum + nch + 1, *gt = gch + kMd5MaxWaves + 1;
    uint64_t *bnd = reinterpret_cast<uint64_t *>(gt + kMd5MaxWaves + 1);
    hipLaunchKernelGGL(k_md5_wsum, dim3((unsigned)nch), dim3(256), 0, s, len, n, csum);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_md5_split, dim3(1), dim3(1024), 0, s, csum, nch, W, gch, gt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_md5_bounds, dim3((W + 1 + 3) / 4), dim3(256), 0, s, len, n, W, csum, gch, gt, bnd);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    bounds = bnd;
  }
  const dim3 g((unsigned)grid), b(64 * kMd5Waves);
#define HC_MD5_LAUNCH(O, L)                                                                                  \
  hipLaunchKernelGGL((k_md5<O, L>), g, b, 0, s, base, off, len, stride, ulen, n, out16, bounds)
  if (off && len)
    HC_MD5_LAUNCH(true, true);
  else if (off)
    HC_MD5_LAUNCH(true, false);
  else if (len)
    HC_MD5_LAUNCH(false, true);
  else
    HC_MD5_LAUNCH(false, false);
#undef HC_MD5_LAUNCH
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
