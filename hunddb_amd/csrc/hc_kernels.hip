// hc_kernels.hip — hand-written gfx950 (CDNA4) kernels of the batched
// block-checksum engine.  CRC-32/IEEE exactly as Go's crc32.ChecksumIEEE,
// applied per block the way /root/reference/utils/crc/crc_util.go:21-33 (stamp)
// and :88-100 (verify) apply it.
//
// Kernels: k_crc_grp (the dominant streaming kernel: 4 KiB-multiple blocks,
// uniform or off/len, blocks handed out per CU), k_crc_fast (uniform 1 KiB
// multiples), k_crc_any (any length / alignment, whole-message CRC), k_frame
// (fused AddCRCsToData), k_unframe (batched ReadFromDisk), k_fill.  The row
// arithmetic they share, as in the streaming kernel k_crc_fast:
// Streaming kernel (k_crc_fast), per wave = one block at a time:
//   * A block of B bytes is B/1024 rows; row j is read by ONE coalesced
//     global_load_dwordx4 (lane l gets bytes 1024j+16l .. +15).  No LDS
//     staging: every byte goes HBM -> VGPR once.
//   * Lane l keeps four Horner streams c_k (word k of its 16 B):
//       c_k <- shift(c_k, 1024) ^ w_k
//     shift(., 1024) is four byte-table lookups (tg) in LDS.  Each table is
//     replicated 32x so lane l reads bank l%32: conflict-free ds_read_b32.
//     The LDS byte address of a lookup is built by ONE v_perm_b32.
//   * Block end: d = shift4^3(c0)^shift4^2(c1)^shift4(c2)^c3 (s4 tables), the
//     lane's placement e = d*x^(8(1012-16l)) mod P as a 32x32 GF(2) mat-vec
//     against 32 lane-constant VGPRs (v_bfe_i32 + v_bitop3), then a DPP/readlane
//     XOR reduction across the 64 lanes.  CRC = xor ^ 0xFFFFFFFF.
//   * Go's init value is the virtual prefix word W0 with shift(W0,4)=~0: in
//     block mode it replaces the stored CRC word (bytes 0..3), which the CRC
//     must not cover anyway.
// General kernel (k_crc_any): any alignment and length (incl. < 4 bytes),
// same row decomposition with the message right-aligned to rows by virtual
// leading zeros; each lane funnel-shifts two aligned 16-B chunks.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "hc_kernels.hpp"
#include "hc_util.hpp"

namespace hc {

namespace {

// The mode word k_seg_stream stores for its batch, in the
// order it is chosen: kSegFallbackGrp, a large batch whose records are all
// 16-B aligned 4 KiB multiples (k_crc_grp's blocks), in any layout: k_crc_grp,
// launched after the combine with this word as its gate; kSegPacked, records
// back to back; kSegGapSmall, sorted records whose gaps are all at most
// kSegSmallGap bytes; kSegGapped, sorted with gaps up to kSegMaxGap (zeroed in
// the stream); kSegFallback, k_crc_any's work inside the combine.
constexpr uint32_t kSegPacked = 0, kSegFallback = 1, kSegGapped = 2, kSegFallbackGrp = 3, kSegGapSmall = 4;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t lds_u32(const uint32_t *lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byte_addr);
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | (uint64_t)uni((uint32_t)v);
}

// 16-B load from an address computed as an integer, as a GLOBAL load.  Through
// a generic pointer hipcc emits flat_load, which also counts on lgkmcnt: every
// later LDS or scalar-load wait then waits for the load too, and a prefetch
// issued before LDS table lookups stops being one.
typedef unsigned int gu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload16(uintptr_t a) {
  const gu32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) gu32x4 *>(a);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 32x32 GF(2) mat-vec: XOR of col[i] over the set bits i of d.
__device__ __forceinline__ uint32_t matvec32(const uint32_t (&col)[32], uint32_t d) {
  uint32_t e = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint32_t m = (uint32_t)((int32_t)(d << (31 - i)) >> 31);  // v_bfe_i32 d, i, 1
    e = __builtin_amdgcn_bitop3_b32(m, col[i], e, 0x6A);      // (m & col) ^ e
  }
  return e;
}

// XOR of v over the 64 lanes (wave-uniform result).
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1032
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm 2301
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16) ^
         __builtin_amdgcn_readlane(v, 32) ^ __builtin_amdgcn_readlane(v, 48);
}

// max of v over the 64 lanes (wave-uniform result)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d));
  return uni(v);
}

// Lane-0 side effects of a wave (CRC word, crc_out, verify atomics) issued with
// exec = lane 0 inside one asm statement.  Written as plain `if (lane == 0)`
// code these become branches around VMEM instructions, and the waitcnt pass
// then assumes the fewest VMEM ops on every path: every wait on a row
// prefetched before the branch turns conservative and also waits for the
// previous block's payload stores.  The asm ops are invisible to that pass;
// that is safe because an extra in-order VMEM op can only make a later
// vmcnt(N) stricter, never looser, and these ops return no data.
__device__ __forceinline__ void lane0_store_u32(uint32_t *p, uint32_t v) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "global_store_dword %1, %2, off\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv)
      : "v"(p), "v"(v)
      : "memory");
}
// per-lane store under an explicit exec mask (asm, so no VMEM instruction sits
// behind a branch; safe for the waitcnt pass for the same reason as above)
__device__ __forceinline__ void lanes_store_u32(uint32_t *p, uint32_t v, uint64_t mask) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, %3\n\t"
      "global_store_dword %1, %2, off\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv)
      : "v"(p), "v"(v), "s"(mask)
      : "memory");
}
__device__ __forceinline__ void lane0_atomic_or(uint32_t *p, uint32_t v) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "global_atomic_or %1, %2, off\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv)
      : "v"(p), "v"(v)
      : "memory");
}
__device__ __forceinline__ void lane0_atomic_umax64(unsigned long long *p, uint64_t v) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "global_atomic_umax_x2 %1, %2, off\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv)
      : "v"(p), "v"(v)
      : "memory");
}
__device__ __forceinline__ void lane0_atomic_umin64(unsigned long long *p, uint64_t v) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "global_atomic_umin_x2 %1, %2, off\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv)
      : "v"(p), "v"(v)
      : "memory");
}

// ---------------------------------------------------------------------------
// k_crc_fast: uniform batches of 16-B aligned blocks whose length is a
// multiple of 1 KiB but not of 4 KiB (4 KiB multiples take k_crc_grp).
// Block b goes to wave b % W (W = every wave of the grid), so all waves sweep
// memory together.  Each wave keeps a ring of kFastRing rows in VGPRs: the row
// just hashed is refilled at once, so kFastRing - 1 rows stay in flight while
// one is hashed.  Round 1 (tools/kbench, profiles/r1/glds/): non-temporal
// loads +17 %, a ring of 4 best, this block order 0-7 % ahead of contiguous
// runs per wave.  The LDS-staged ring it was measured against, the timing-only
// build and the round-1 off/len path are in git history (tools/ab_hc_kernels.hip,
// up to commit 61a2e0e).
constexpr int kFastRing = 4;

// Row load, 16 B per lane, non-temporal (the blocks are read once).
__device__ __forceinline__ uint4 load_row(const uint8_t *row, uint32_t lane) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(row + lane * 16u));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// The replicated LDS tables every CRC kernel uses: the row-shift tables (main
// region: table k, byte v, replica r at (k>>1)<<16 | v<<8 | (k&1)<<7 | r<<2,
// 32 replicas, conflict-free) and the 4-byte shift tables (kLdsMainBytes +
// (k*256 + v)*16 + r*4, 4 replicas).
__device__ __forceinline__ void fill_crc_tables(uint32_t *lds, const DeviceTables *tables, uint32_t tid,
                                                uint32_t nthreads) {
  const uint32_t *tg = &tables->tg[0][0];
  for (uint32_t q = tid; q < kLdsMainBytes / 16; q += nthreads) {
    const uint32_t a = q * 16;
    const uint32_t k = ((a >> 16) << 1) | ((a >> 7) & 1u);
    const uint32_t v = tg[k * 256 + ((a >> 8) & 255u)];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + a) = make_uint4(v, v, v, v);
  }
  const uint32_t *s4 = &tables->s4[0][0];
  for (uint32_t q = tid; q < kLdsS4Bytes / 16; q += nthreads) {
    const uint32_t v = s4[q];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + kLdsMainBytes + q * 16) = make_uint4(v, v, v, v);
  }
}

__global__ __launch_bounds__(kFastThreads) void k_crc_fast(const uint8_t *base, uint64_t stride, uint32_t ulen,
                                                          uint32_t flags, uint64_t nblocks,
                                                          uint32_t *__restrict__ crc_out,
                                                          uint32_t *__restrict__ bad_bitmap,
                                                          unsigned long long *__restrict__ first_bad,
                                                          const DeviceTables *__restrict__ tables) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  fill_crc_tables(lds, tables, tid, kFastThreads);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  const uint32_t w0 = tables->w0;
  __syncthreads();

  const uint32_t r4 = (lane & 31u) << 2;
  const uint32_t B0 = r4, B1 = r4 | 128u, B2 = 65536u | r4, B3 = 65536u | 128u | r4;
  const uint32_t S4base = kLdsMainBytes + ((lane & 3u) << 2);
  const bool msg = (flags & kFlagMessages) != 0;

  // c <- shift(c, 1024) ^ w : four conflict-free lookups, one v_perm each.
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(c, B0, 0x0c020400u));
    const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(c, B1, 0x0c020500u));
    const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(c, B2, 0x0c020600u));
    const uint32_t t3 = lds_u32(lds, __builtin_amdgcn_perm(c, B3, 0x0c020700u));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, S4base + ((x & 255u) << 4));
    const uint32_t t1 = lds_u32(lds, S4base + 4096u + (((x >> 8) & 255u) << 4));
    const uint32_t t2 = lds_u32(lds, S4base + 8192u + (((x >> 16) & 255u) << 4));
    const uint32_t t3 = lds_u32(lds, S4base + 12288u + ((x >> 24) << 4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };

  const uint32_t wave = uni(tid >> 6);
  const uint64_t step = (uint64_t)gridDim.x * kFastWaves;  // block b -> wave b % step
  const uint32_t rows = ulen >> 10;

  // ---- producer: cursor over this wave's blocks and the rows of the current one
  uint64_t pb = (uint64_t)blockIdx.x * kFastWaves + wave;
  if (pb >= nblocks) return;
  const uint8_t *pptr = base + pb * stride;
  uint32_t prow = 0;
  bool pvalid = true;
  // Each ring slot carries the wave-uniform tag of the row it holds.  The load
  // is unconditional (past the wave's last row it re-reads that row, tagged
  // invalid) so hipcc's wait counting stays exact: vmcnt(kFastRing-1).
  struct Tag {
    uint64_t blk;
    const uint8_t *ptr;
    uint32_t row;
    bool valid;
  };
  auto load_next = [&](Tag &t) -> uint4 {
    const uint4 v = load_row(pptr + (size_t)prow * kRowBytes, lane);
    t.valid = pvalid;
    t.blk = pb;
    t.ptr = pptr;
    t.row = prow;
    if (pvalid && ++prow == rows) {
      if (pb + step < nblocks) {
        pb += step;
        pptr = base + pb * stride;
        prow = 0;
      } else {  // park on the last row
        pvalid = false;
        prow = rows - 1;
      }
    }
    return v;
  };
  uint4 ring[kFastRing];
  Tag tag[kFastRing];
#pragma unroll
  for (int u = 0; u < kFastRing; u++) ring[u] = load_next(tag[u]);

  // ---- consumer
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, stored = 0;
  bool reported = false;  // wave-uniform: this wave already lowered first_bad
  for (;;) {
#pragma unroll
    for (int u = 0; u < kFastRing; u++) {
      // consume slot u, then refill it (same registers: no copies)
      const Tag t = tag[u];
      uint4 v = ring[u];
      if (t.row == 0) {
        if (lane == 0) {
          stored = v.x;
          v.x = msg ? (v.x ^ 0xFFFFFFFFu) : w0;
        }
        c0 = v.x;
        c1 = v.y;
        c2 = v.z;
        c3 = v.w;
      } else {
        c0 = row_step(c0, v.x);
        c1 = row_step(c1, v.y);
        c2 = row_step(c2, v.z);
        c3 = row_step(c3, v.w);
      }
      ring[u] = load_next(tag[u]);
      if (t.row + 1 == rows) {
        const uint32_t d = shift4(shift4(shift4(c0, c1), c2), c3);
        const uint32_t crc = wave_xor(matvec32(col, d)) ^ 0xFFFFFFFFu;
        if (lane == 0) {
          const uint64_t cb = t.blk;
          if (crc_out) crc_out[cb] = crc;
          if (flags & kFlagStamp) *const_cast<uint32_t *>(reinterpret_cast<const uint32_t *>(t.ptr)) = crc;
          if (first_bad && stored != crc) {
            if (bad_bitmap)
              __hip_atomic_fetch_or(&bad_bitmap[cb >> 5], 1u << (cb & 31), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
            if (!reported)
              __hip_atomic_fetch_min(first_bad, (unsigned long long)cb, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        // a wave meets its blocks in increasing order: after its first bad
        // block, further first_bad atomics cannot lower the minimum (and on a
        // batch of all-bad blocks would serialise every wave on one address)
        if (first_bad && uni(stored) != crc) reported = true;
        if (!tag[(u + 1) % kFastRing].valid) return;  // the wave's last block is done
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_crc_grp: the streaming kernel for blocks of 4 KiB multiples with the
// k_crc_uni group structure, for uniform batches and off/len batches alike,
// with the blocks dealt to waves by a per-workgroup hand-out.
//   * Workgroup g owns the chunks of C = 2^lg_chunk consecutive blocks
//     c*G + g (G = grid): all workgroups sweep memory together, and the CRC
//     words / bitmap bits of one chunk are written by one CU (one XCD's L2:
//     a 128-B line of crc_out is 32 blocks).
//   * Inside the workgroup the blocks are handed out one at a time by an LDS
//     counter (ds_add_rtn, lane 0, once per block, its value used one block
//     later).  Mixed 4/8/16 KiB batches (configs[2]) then keep every wave of a
//     CU busy to the end; a static deal leaves per-wave byte totals ~3 % apart
//     (sd), and the slowest wave sets the kernel time.
//   * off/len metadata of the block after next is read by a buffer load issued
//     before each iteration's first row refill, so it is complete by the time
//     the next refill's row has been waited for (in-order vmcnt): no wait of
//     its own, no scalar load in flight across the LDS lookups.  It is issued
//     every iteration (the same entry again between block ends) so no VMEM
//     instruction sits behind a branch.
//   * A block that is not 16-B aligned or whose length is not a positive
//     multiple of 4096 costs one group of dummy rows (re-reads of the current
//     group, never stored) and is left to k_crc_any (fast_mask 4095).
//   * kXcd: workgroup g runs on XCD g % 8; the chunk slots are renumbered so
//     that each XCD's workgroups own neighbouring chunks (grp_xcd decides).
//   * Paired placement (round 4): a wave finalises its blocks two at a time.
//     Lane l's placement M_l (shift by 1012 - 16 l bytes) is shift(512) of
//     lane l+32's, so block A folds lanes l and l+32 into lane l+32 (d_{l+32} ^
//     shift(d_l, 512)) and block B into lane l (d_l ^ shift(d_{l+32}, -512)):
//     one 4-lookup shift (lanes 0-31 forward, 32-63 inverse, 8 KiB of LDS), a
//     v_permlane32_swap, ONE 32x32 mat-vec for both, and the XORs of the lower
//     and upper halves.  The block waiting for a partner keeps d in a VGPR; the
//     wave's last odd block is finalised alone.  Against one mat-vec a block:
//     SQ_INSTS_VALU -11.5 % at 1M x 4 KiB, +0.65 points at 4 KiB and +0.17 at
//     8 KiB over five and four same-box A/B pairs (profiles/r4/r4a, r4b, r4c).
// The variants measured against this one before round 4 (static deal, batched
// refills, nibble finalise tables, timing-only build) are in git history
// (tools/ab_hc_kernels.hip, up to commit 61a2e0e).
// The body, a device function called by the k_crc_grp kernel below only.  (Round
// 5 also ran it inside k_seg_combine, ahead of crc_any_body behind a runtime
// mode: hipcc then left the implicit-argument pointer that gridDim.x is read
// through written on this body's path only, and the plain fallback read it from
// a stale SGPR pair -- the r5d illegal address; DESIGN.md 4.2a,
// tests/test_isa_sgpr_defs.py.  The packed-record stream's k_crc_grp fallback is
// a separate gated launch.)  `lds` holds kFastLdsBytes of tables and the 8 KiB
// sh512 table after them.
template <bool kArrays, bool kXcd>
__device__ __forceinline__ void crc_grp_body(uint32_t *lds, uint32_t &s_next, const uint8_t *base,
                                             const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
                                             uint64_t stride, uint32_t ulen, uint32_t flags, uint64_t nblocks,
                                             uint32_t lg_chunk, uint32_t *__restrict__ crc_out,
                                             uint32_t *__restrict__ bad_bitmap,
                                             unsigned long long *__restrict__ first_bad,
                                             const DeviceTables *__restrict__ tables,
                                             unsigned long long *__restrict__ skip_slot, uint64_t skip_tag) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  fill_crc_tables(lds, tables, tid, kFastThreads);
  for (uint32_t q = tid; q < 2048; q += kFastThreads) lds[kFastLdsBytes / 4 + q] = (&tables->sh512[0][0][0])[q];
  if (tid == 0) s_next = 3 * kFastWaves;  // indices 0 .. 3W-1 are dealt statically below
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  const uint32_t w0 = tables->w0;
  __syncthreads();

  const uint32_t r4 = (lane & 31u) << 2;
  const uint32_t B0 = r4, B1 = r4 | 128u, B2 = 65536u | r4, B3 = 65536u | 128u | r4;
  const uint32_t S4base = kLdsMainBytes + ((lane & 3u) << 2);
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(c, B0, 0x0c020400u));
    const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(c, B1, 0x0c020500u));
    const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(c, B2, 0x0c020600u));
    const uint32_t t3 = lds_u32(lds, __builtin_amdgcn_perm(c, B3, 0x0c020700u));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, S4base + ((x & 255u) << 4));
    const uint32_t t1 = lds_u32(lds, S4base + 4096u + (((x >> 8) & 255u) << 4));
    const uint32_t t2 = lds_u32(lds, S4base + 8192u + (((x >> 16) & 255u) << 4));
    const uint32_t t3 = lds_u32(lds, S4base + 12288u + ((x >> 24) << 4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };

  // paired placement: lanes 0-31 shift by 512 bytes, lanes 32-63 by -512
  const uint32_t PHbase = kFastLdsBytes + ((lane >> 5) << 12);
  auto pshift = [&](uint32_t y) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, PHbase + ((y & 255u) << 2));
    const uint32_t t1 = lds_u32(lds, PHbase + 1024u + (((y >> 8) & 255u) << 2));
    const uint32_t t2 = lds_u32(lds, PHbase + 2048u + (((y >> 16) & 255u) << 2));
    const uint32_t t3 = lds_u32(lds, PHbase + 3072u + ((y >> 24) << 2));
    return xor3(t0, t1, t2) ^ t3;
  };

  const uint32_t wave = uni(tid >> 6);
  const uint64_t G = gridDim.x;
  // kXcd: each XCD's workgroups own neighbouring chunk slots (G a multiple of 8)
  const uint64_t wg = kXcd && (G & 7u) == 0 ? (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const uint32_t cmask = (1u << lg_chunk) - 1u;
  // k-th block of this workgroup's sequence, increasing in k: the first one
  // past the batch ends the wave (a per-workgroup rotation inside the chunks
  // was measured -- no gain -- and would break that rule on a partial chunk)
  auto blk_of = [&](uint32_t k) -> uint64_t { return (((uint64_t)(k >> lg_chunk) * G + wg) << lg_chunk) | (k & cmask); };
  const bool msg = (flags & kFlagMessages) != 0;

  // metadata -> (group pointer, group count, skip)
  struct Blk {
    uint64_t i;
    const uint8_t *p;
    uint32_t groups;
    bool valid, skip;
  };
  auto make_blk = [&](uint64_t i, uint64_t o, uint32_t l) {
    Blk r;
    r.i = i;
    r.valid = i < nblocks;
    r.p = base + o;
    r.groups = l >> 12;
    r.skip = kArrays && (((((uintptr_t)base + o) & 15u) != 0) || (l & 4095u) != 0 || l == 0);
    return r;
  };
  auto meta_sync = [&](uint64_t i) {  // prologue only
    if constexpr (!kArrays) return make_blk(i, i * stride, ulen);
    const uint64_t ic = i < nblocks ? i : 0;
    return make_blk(i, offs[ic], lens[ic]);
  };
  // the block after next: its metadata as a buffer load (vmcnt-ordered)
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 m_o = {0, 0};
  uint32_t m_l = 0;
  auto meta_issue = [&](uint64_t i) {
    if constexpr (kArrays) {
      const uint64_t ic = i < nblocks ? i : 0;  // (wave-uniform) descriptors based at the entry
      const __amdgpu_buffer_rsrc_t ro =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(offs + ic), 0, 8, 0x00020000);
      const __amdgpu_buffer_rsrc_t rl =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(lens + ic), 0, 4, 0x00020000);
      m_o = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(ro, 0, 0, 0));
      m_l = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rl, 0, 0, 0);
    }
  };

  uint32_t k0 = wave, k1 = kFastWaves + wave, k2 = 2 * kFastWaves + wave;
  const uint64_t i0 = blk_of(k0);
  if (i0 >= nblocks) return;
  Blk cur = meta_sync(i0);
  Blk n1 = meta_sync(blk_of(k1));
  uint64_t i2 = blk_of(k2);
  uint32_t k3v = 0;  // VGPR: the LDS hand-out result, read one block end later
  meta_issue(i2);
  // the group the row registers hold; a skipped first block reads 4 KiB of the
  // constant image instead (always mapped, never consumed)
  const uint8_t *gp = cur.skip ? reinterpret_cast<const uint8_t *>(tables) : cur.p;
  static_assert(sizeof(DeviceTables) >= 4096, "dummy group reads 4 KiB of the table image");
  uint32_t g = 0, gc = cur.skip ? 1u : cur.groups;
  uint4 q0 = load_row(gp, lane), q1 = load_row(gp + 1024, lane), q2 = load_row(gp + 2048, lane),
        q3 = load_row(gp + 3072, lane);
  if (lane == 0) k3v = atomicAdd(&s_next, 1u);
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, stored = 0;
  uint64_t reported = ~0ull;  // wave-uniform: lowest block this wave has put into first_bad
  // a block's outputs: CRC word, stamp, verify bitmap / first_bad
  auto emit = [&](uint64_t b, const uint8_t *p, uint32_t st, uint32_t crc) {
    if (crc_out) lane0_store_u32(crc_out + b, crc);
    if (flags & kFlagStamp) lane0_store_u32(const_cast<uint32_t *>(reinterpret_cast<const uint32_t *>(p)), crc);
    const bool bad = st != crc;
    if (first_bad && bad) {
      if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
      // blocks arrive in increasing order: one atomic per wave (a batch of
      // all-bad blocks would otherwise serialise every wave on one word)
      if (b < reported) lane0_atomic_umin64(first_bad, b);
      reported = b < reported ? b : reported;
    }
  };
  // the finalised block waiting for a partner (its lane-combined streams)
  bool pend = false;
  uint32_t pd = 0, pst = 0;
  uint64_t pi = 0;
  const uint8_t *pp = nullptr;
  for (;;) {
    const bool last = g + 1 == gc;
    // refills: this block's next group, or the next block's first group (a
    // skipped or missing next block: this group again, never consumed)
    const uint8_t *np = !last ? gp + 4096 : ((n1.valid && !n1.skip) ? n1.p : gp);
    if (g == 0) {
      uint4 v = q0;
      if (lane == 0) {
        stored = v.x;
        v.x = msg ? (v.x ^ 0xFFFFFFFFu) : w0;
      }
      c0 = v.x;
      c1 = v.y;
      c2 = v.z;
      c3 = v.w;
    } else {
      c0 = row_step(c0, q0.x);
      c1 = row_step(c1, q0.y);
      c2 = row_step(c2, q0.z);
      c3 = row_step(c3, q0.w);
    }
    // consumer's next block (the rows the refills below fetch)
    const Blk nxt = n1;
    if (last) {
      // n1 <- n2 (its metadata arrived with the row just waited for), n2 <- hand-out
      if constexpr (kArrays) {
        const uint64_t o = ((uint64_t)uni(m_o.y) << 32) | (uint64_t)uni(m_o.x);
        n1 = make_blk(i2, o, uni(m_l));
      } else {
        n1 = make_blk(i2, i2 * stride, ulen);
      }
      const uint32_t k3 = uni(k3v);
      if (lane == 0) k3v = atomicAdd(&s_next, 1u);
      i2 = blk_of(k3);
    }
    // Each refill right after its row's hash (the sched_barriers keep hipcc
    // from pairing them two rows late: +0.3-0.8 %); issuing a group's four
    // refills together after its last row, as a plain read stream does, was
    // 0.3-1 % slower (profiles/r2/ab_refill/).
    meta_issue(i2);
    q0 = load_row(np, lane);
    __builtin_amdgcn_sched_barrier(0);
    c0 = row_step(c0, q1.x);
    c1 = row_step(c1, q1.y);
    c2 = row_step(c2, q1.z);
    c3 = row_step(c3, q1.w);
    __builtin_amdgcn_sched_barrier(0);
    q1 = load_row(np + 1024, lane);
    __builtin_amdgcn_sched_barrier(0);
    c0 = row_step(c0, q2.x);
    c1 = row_step(c1, q2.y);
    c2 = row_step(c2, q2.z);
    c3 = row_step(c3, q2.w);
    __builtin_amdgcn_sched_barrier(0);
    q2 = load_row(np + 2048, lane);
    __builtin_amdgcn_sched_barrier(0);
    c0 = row_step(c0, q3.x);
    c1 = row_step(c1, q3.y);
    c2 = row_step(c2, q3.z);
    c3 = row_step(c3, q3.w);
    __builtin_amdgcn_sched_barrier(0);
    q3 = load_row(np + 3072, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (last) {  // block cur is complete
      if (!cur.skip) {
        const uint32_t d = shift4(shift4(shift4(c0, c1), c2), c3);
        if (!pend) {  // wait for a partner
          pd = d;
          pst = uni(stored);
          pi = cur.i;
          pp = cur.p;
          pend = true;
        } else {
          // two blocks, one placement: A (pending) is folded into lanes 32-63
          // (d_j ^ shift(d_{j-32}, 512): lane j's placement covers both), B
          // (this one) into lanes 0-31 (d_l ^ shift(d_{l+32}, -512)); one
          // 32x32 mat-vec, then the lower and upper halves' XORs
          const bool lo = lane < 32;
          const uint32_t z = pshift(lo ? pd : d);
          const auto sw = __builtin_amdgcn_permlane32_swap(z, z, false, false);
          const uint32_t x = (lo ? d : pd) ^ (lo ? sw[1] : sw[0]);
          uint32_t v = matvec32(col, x);
          v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
          v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
          v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
          v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
          const uint32_t crc_b = __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16) ^ 0xFFFFFFFFu;
          const uint32_t crc_a = __builtin_amdgcn_readlane(v, 32) ^ __builtin_amdgcn_readlane(v, 48) ^ 0xFFFFFFFFu;
          emit(pi, pp, pst, crc_a);
          emit(cur.i, cur.p, uni(stored), crc_b);
          pend = false;
        }
      } else if (kArrays && skip_slot && skip_tag) {  // left to the k_crc_any sweep: tell it once per wave
        // a relaxed load first: once one wave has raised the word the others
        // skip their atomic (a batch whose blocks all go to the sweep put one
        // same-address atomic per wave on it, serialised at the L2: 45 us at
        // 4096 blocks, profiles/r4/r4v/)
        if (__hip_atomic_load(skip_slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < skip_tag)
          lane0_atomic_umax64(skip_slot, skip_tag);
        skip_tag = 0;
      }
      if (!nxt.valid) {
        if (pend) emit(pi, pp, pst, wave_xor(matvec32(col, pd)) ^ 0xFFFFFFFFu);  // no partner left
        return;
      }
      cur = nxt;
      g = 0;
      gc = cur.skip ? 1u : cur.groups;
      gp = np;
    } else {
      g++;
      gp = np;
    }
  }
}

template <bool kArrays, bool kXcd = false>
__global__ __launch_bounds__(kFastThreads) void k_crc_grp(const uint8_t *base, const uint64_t *__restrict__ offs,
                                                         const uint32_t *__restrict__ lens, uint64_t stride,
                                                         uint32_t ulen, uint32_t flags, uint64_t nblocks,
                                                         uint32_t lg_chunk, uint32_t *__restrict__ crc_out,
                                                         uint32_t *__restrict__ bad_bitmap,
                                                         unsigned long long *__restrict__ first_bad,
                                                         const DeviceTables *__restrict__ tables,
                                                         unsigned long long *__restrict__ skip_slot = nullptr,
                                                         uint64_t skip_tag = 0,
                                                         const uint32_t *__restrict__ gate = nullptr) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4 + 2048];
  __shared__ uint32_t s_next;  // next hand-out index of this workgroup's block sequence
  if (gate && *gate != kSegFallbackGrp) return;  // the packed-record stream's fallback only (launch_seg)
  crc_grp_body<kArrays, kXcd>(lds, s_next, base, offs, lens, stride, ulen, flags, nblocks, lg_chunk, crc_out,
                              bad_bitmap, first_bad, tables, skip_slot, skip_tag);
}

// ---------------------------------------------------------------------------
// General kernel (k_crc_any): any alignment, any length (incl. < 4 bytes),
// block or whole-message mode.  One wave per block, 16 waves per CU, the same
// replicated LDS tables and per-lane Horner streams as the streaming kernel.
//
// The message M = payload (block mode: bytes [4, len); message mode: all) is
// processed as the virtual message  zeros(z) || W0 || M  of `rows` 1 KiB
// rows (raw() ignores leading zeros; W0 is Go's init).  Row r, lane l covers
// payload offsets s_r + 16l .. +15 with s_r = 1024r - z - 4.  Every row has
// the same misalignment m = (P - z - 4) mod 16, so each lane loads the two
// aligned 16-B chunks around its window (the second one is the neighbour's
// first: an L1 hit) and funnel-shifts them by m.  Chunks that do not overlap
// [P, P+Lp) are not loaded (no byte outside the block is touched); bytes at
// negative offsets are replaced by zeros / W0.
//
// only_nonfast: the wave fetches the metadata of 64 blocks with one
// coalesced load, ballots which of them the streaming kernel skipped, and
// processes only those (so a batch the streaming kernel fully covered costs
// one metadata sweep, not a per-block scan).
// 16 bytes starting at byte m = 4q + rb of the 32-byte pair (a, b): one
// uniform switch per row, named registers only (no array -> no scratch).
__device__ __forceinline__ uint4 funnel16(const uint4 a, const uint4 b, uint32_t q, uint32_t rb) {
  switch (q) {
    case 0:
      return make_uint4(__builtin_amdgcn_alignbyte(a.y, a.x, rb), __builtin_amdgcn_alignbyte(a.z, a.y, rb),
                        __builtin_amdgcn_alignbyte(a.w, a.z, rb), __builtin_amdgcn_alignbyte(b.x, a.w, rb));
    case 1:
      return make_uint4(__builtin_amdgcn_alignbyte(a.z, a.y, rb), __builtin_amdgcn_alignbyte(a.w, a.z, rb),
                        __builtin_amdgcn_alignbyte(b.x, a.w, rb), __builtin_amdgcn_alignbyte(b.y, b.x, rb));
    case 2:
      return make_uint4(__builtin_amdgcn_alignbyte(a.w, a.z, rb), __builtin_amdgcn_alignbyte(b.x, a.w, rb),
                        __builtin_amdgcn_alignbyte(b.y, b.x, rb), __builtin_amdgcn_alignbyte(b.z, b.y, rb));
    default:
      return make_uint4(__builtin_amdgcn_alignbyte(b.x, a.w, rb), __builtin_amdgcn_alignbyte(b.y, b.x, rb),
                        __builtin_amdgcn_alignbyte(b.z, b.y, rb), __builtin_amdgcn_alignbyte(b.w, b.z, rb));
  }
}

// Buffer load of 16 bytes at byte offset `voff` of the range `r`: an offset at
// or past the range's end returns zeros WITHOUT touching memory (the buffer
// range check).  That is how k_crc_any predicates its loads: no branch around
// any VMEM instruction, so hipcc's vmcnt counting stays exact across the
// software pipeline.  aux 2 = nt (read-once data).
__device__ __forceinline__ uint4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 2));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_range(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
// Buffer store of one word per lane: lanes whose offset is at or past the
// range's end store nothing.  A compiler-visible VMEM op issued on every path,
// so the waitcnt pass counts it exactly (an asm store after a prefetch makes
// the prefetch's wait also wait for the next one).
__device__ __forceinline__ void buf_store_u32(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, 0, 0);
}

// Pipelined per wave over its messages (blocks in block mode): the edge rows
// of message i+1 (and its stored word) are loaded while message i is
// finalised, and message i's first body batch (issued only when the message
// has body rows) together with its edge rows, during the previous message's
// finalise (profiles/r1/s5/kmsg_variants2.txt: best or within 1 % of the best
// on config 5b, equal-size messages and 4092-B off/len blocks).  Body rows go
// kAnyBatch at a time.  Windows of 64 messages are handed out like k_crc_grp's
// blocks: workgroup g owns the chunks of 2^lg_chunk consecutive windows
// c*G + g, its waves take windows one at a time from an LDS counter (+1.5-4.5 %
// over one static run per wave, profiles/r2/any/).  kSmallLanes (whole-message
// batches): records of <= 1020 bytes are hashed one per lane (below).  The
// measured alternatives (static runs, other batch sizes, issue orders, the
// timing-only build) are in git history (tools/ab_hc_kernels.hip, up to 61a2e0e).
constexpr int kAnyBatch = 4;
// The body, a device function: the k_crc_any kernel below, and k_seg_combine
// for a batch the packed-record stream did not take (the fallback in the same
// launch).  `lds` holds kFastLdsBytes of tables and one word after them, the
// workgroup's window counter.
template <bool kSmallLanes>
__device__ __forceinline__ void crc_any_body(
    uint32_t *lds, const uint8_t *base, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
    uint64_t stride, uint32_t ulen, uint32_t flags, uint64_t nblocks, uint32_t fast_mask, uint32_t lg_chunk,
    uint32_t *__restrict__ crc_out, uint32_t *__restrict__ bad_bitmap,
    unsigned long long *__restrict__ first_bad, const DeviceTables *__restrict__ tables,
    const unsigned long long *skip_slot, uint64_t skip_tag) {
  uint32_t &s_next = lds[kFastLdsBytes / 4];
  // the sweep after k_crc_grp: no block was left to it (Batch::skip_slot)
  if (fast_mask && skip_slot &&
      __hip_atomic_load(skip_slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < skip_tag)
    return;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = uni(tid >> 6);
  const uint64_t b1 = nblocks;
  const uint64_t G = gridDim.x, wg = blockIdx.x;
  const uint32_t cmask = (1u << lg_chunk) - 1u;
  // windows of 64 messages, fewer on small batches so that every wave gets one
  // (a wave hashes its window's records one after another: 4096 records in
  // 64-message windows kept 64 of 4096 waves busy, 42-82 us, profiles/r4/r4t/)
  uint32_t lgw = 6;
  while (lgw > 0 && (b1 >> lgw) < G * kFastWaves) lgw--;
  const uint32_t W = 1u << lgw;
  // first message of the workgroup's k-th window (increasing in k)
  auto win_of = [&](uint32_t k) -> uint64_t {
    return ((((uint64_t)(k >> lg_chunk) * G + wg) << lg_chunk) | (k & cmask)) << lgw;
  };
  if (tid == 0) s_next = kFastWaves;
  // fast_mask != 0 (the sweep after a streaming kernel): look for work before
  // the 144 KiB table fill -- a batch the streaming kernel fully covered costs
  // one metadata read per block and no fill (kbench2: 10 us -> a few).  The
  // workgroup checks exactly the messages it will own.
  if (fast_mask) {
    bool any = false;
    for (uint32_t kk = wave;; kk += kFastWaves) {
      const uint64_t g0 = win_of(kk);
      if (g0 >= b1 || any) break;
      const uint64_t j = g0 + lane;
      const bool in = lane < W && j < b1;
      const uint64_t oj = in ? (offs ? offs[j] : j * stride) : 0;
      const uint32_t lj = in ? (lens ? lens[j] : ulen) : 0;
      const bool fast = (((uintptr_t)base + oj) & 15u) == 0 && (lj & fast_mask) == 0 && lj != 0;
      any = __ballot(in && !fast) != 0;
    }
    if (!__syncthreads_or(any)) return;
  }
  fill_crc_tables(lds, tables, tid, kFastThreads);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  const uint32_t w0 = tables->w0;
  __syncthreads();

  const uint32_t r4 = (lane & 31u) << 2;
  const uint32_t B0 = r4, B1 = r4 | 128u, B2 = 65536u | r4, B3 = 65536u | 128u | r4;
  const uint32_t S4base = kLdsMainBytes + ((lane & 3u) << 2);
  const bool msg = (flags & kFlagMessages) != 0;
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(c, B0, 0x0c020400u));
    const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(c, B1, 0x0c020500u));
    const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(c, B2, 0x0c020600u));
    const uint32_t t3 = lds_u32(lds, __builtin_amdgcn_perm(c, B3, 0x0c020700u));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, S4base + ((x & 255u) << 4));
    const uint32_t t1 = lds_u32(lds, S4base + 4096u + (((x >> 8) & 255u) << 4));
    const uint32_t t2 = lds_u32(lds, S4base + 8192u + (((x >> 16) & 255u) << 4));
    const uint32_t t3 = lds_u32(lds, S4base + 12288u + ((x >> 24) << 4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };

  // ---- small records, one per lane (kSmallLanes, whole-message mode) --------
  // A window's records of <= 1020 bytes (one row) are hashed lane-parallel:
  // lane k takes record g+k (its metadata is already in this lane) and runs
  // the Horner chain c <- shift4(c) ^ V_i over the 4-byte words of the
  // virtual message zeros(z) || W0 || M (z = -L mod 4), then
  // crc = shift4(c) ^ ~0 (the 4-byte placement of the row kernels' last lane).
  // Loads are the aligned 16-B chunks of [Q, Q + T) (Q = P - z - 4), four in
  // flight per lane; a chunk that does not overlap the record reads 16 bytes
  // of the constant table image instead (only prefix bytes, masked, or bytes
  // past the end, unused, come from such a chunk), so no byte outside the
  // record's own aligned chunks is touched and no load sits behind a branch.
  constexpr uint32_t kSmallMax = kRowBytes - 4;
  auto small_lanes = [&](uint64_t m, uint64_t oj, uint32_t lj, uint64_t g0) {
    const bool act = (m >> lane) & 1u;
    const uint32_t L = act ? lj : 0u;
    const uintptr_t P = (uintptr_t)base + (act ? oj : 0u);
    const uint32_t z = (4u - (L & 3u)) & 3u;
    const uint32_t T = z + 4u + L;  // virtual bytes, a multiple of 4
    const uint32_t nw = T >> 2;
    const uintptr_t Q = P - z - 4u;
    const uintptr_t Qa = Q & ~(uintptr_t)15;
    const uint32_t mq = (uint32_t)(Q & 15u), qw = mq >> 2, rb = mq & 3u;
    const uint32_t nch = (mq + T + 15u) >> 4;
    uint32_t mx = 0;  // wave max of nch (<= 66) by ballot
    for (uint32_t bb = 64; bb; bb >>= 1)
      if (__ballot(act && nch >= mx + bb)) mx += bb;
    const uintptr_t safe = (uintptr_t)tables;
    auto ld = [&](uint32_t c) -> uint4 {
      const uintptr_t X = Qa + 16u * c;
      const bool in = act && L > 0 && X + 16u > P && X < P + L;
      // plain (cached) load: records packed back to back share lines that the
      // next chunks of the neighbouring lanes read again
      return gload16(in ? X : safe);
    };
    auto sel = [&](uint32_t a, uint32_t b, uint32_t c2, uint32_t d) { return qw == 0 ? a : qw == 1 ? b : qw == 2 ? c2 : d; };
    // 16 bytes at byte mq of the 32-byte pair (a, b), mq per lane
    auto fun = [&](const uint4 &a, const uint4 &b) {
      const uint32_t w0_ = sel(a.x, a.y, a.z, a.w), w1_ = sel(a.y, a.z, a.w, b.x), w2_ = sel(a.z, a.w, b.x, b.y),
                     w3_ = sel(a.w, b.x, b.y, b.z), w4_ = sel(b.x, b.y, b.z, b.w);
      return make_uint4(__builtin_amdgcn_alignbyte(w1_, w0_, rb), __builtin_amdgcn_alignbyte(w2_, w1_, rb),
                        __builtin_amdgcn_alignbyte(w3_, w2_, rb), __builtin_amdgcn_alignbyte(w4_, w3_, rb));
    };
    const uint64_t Y = (uint64_t)w0 << 32;
    uint32_t c = 0;
    auto step = [&](uint32_t i, uint32_t w, bool head) {
      if (head) {  // words 0 and 1 may hold the prefix: zeros, then W0 (as the edge rows do)
        const int32_t d = -((int32_t)(4u * i) - (int32_t)z - 4);
        const uint32_t dm = d <= 0 ? 0xFFFFFFFFu : (d >= 4 ? 0u : 0xFFFFFFFFu << (8 * d));
        const uint32_t wv = (d >= 1 && d <= 8) ? (uint32_t)(Y >> (64 - 8 * d)) : 0u;
        w = (w & dm) | wv;
      }
      const uint32_t nc = i == 0 ? w : shift4(c, w);
      c = i < nw ? nc : c;
    };
    uint4 A0 = ld(0), A1 = ld(1), A2 = ld(2), A3 = ld(3);
    for (uint32_t k = 0; k < mx; k += 4) {
      // chunk pair (k+j, k+j+1) gives words 4(k+j) .. +3; chunk k+j is
      // reloaded with chunk k+j+4 right after its last use
      const bool head = k == 0;
      uint4 f = fun(A0, A1);
      A0 = ld(k + 4);
      step(4 * k + 0, f.x, head);
      step(4 * k + 1, f.y, head);
      step(4 * k + 2, f.z, false);
      step(4 * k + 3, f.w, false);
      f = fun(A1, A2);
      A1 = ld(k + 5);
      step(4 * k + 4, f.x, false);
      step(4 * k + 5, f.y, false);
      step(4 * k + 6, f.z, false);
      step(4 * k + 7, f.w, false);
      f = fun(A2, A3);
      A2 = ld(k + 6);
      step(4 * k + 8, f.x, false);
      step(4 * k + 9, f.y, false);
      step(4 * k + 10, f.z, false);
      step(4 * k + 11, f.w, false);
      f = fun(A3, A0);
      A3 = ld(k + 7);
      step(4 * k + 12, f.x, false);
      step(4 * k + 13, f.y, false);
      step(4 * k + 14, f.z, false);
      step(4 * k + 15, f.w, false);
    }
    asm volatile("" ::"v"(A0.x), "v"(A1.x), "v"(A2.x), "v"(A3.x));  // consume the last loads here
    const uint32_t crc = shift4(c, 0u) ^ 0xFFFFFFFFu;
    if (crc_out) lanes_store_u32(crc_out + g0 + lane, crc, m);
  };

  // ---- message cursor ------------------------------------------------------
  // The metadata of 64 messages g .. g+63 sits one per lane (one coalesced
  // load); `todo` ballots the ones this kernel must do (only_nonfast: those
  // the streaming kernel skipped).  Entries are read with v_readlane.
  uint64_t g = win_of(wave), todo = 0;
  bool loaded = false;
  uint32_t wo_lo = 0, wo_hi = 0, wl = 0;
  uint32_t knv = 0;  // LDS hand-out result for the next window, read one window later
  if (lane == 0) knv = atomicAdd(&s_next, 1u);
  struct Msg {
    uint64_t blk;
    const uint8_t *p;  // block / message start
    uint32_t l;
    bool valid;
  };
  auto next = [&](Msg &mm) {
    for (;;) {
      if (todo) {
        const uint32_t k = (uint32_t)__builtin_ctzll(todo);
        todo &= todo - 1;
        // readlane returns int: cast each half to uint32_t BEFORE widening, or
        // a low word >= 2^31 sign-extends into the high word (a wild address)
        const uint32_t o_lo = (uint32_t)__builtin_amdgcn_readlane(wo_lo, k);
        const uint32_t o_hi = (uint32_t)__builtin_amdgcn_readlane(wo_hi, k);
        mm.blk = g + k;
        mm.p = base + (((uint64_t)o_hi << 32) | (uint64_t)o_lo);
        mm.l = (uint32_t)__builtin_amdgcn_readlane(wl, k);
        mm.valid = true;
        return;
      }
      if (loaded) {
        g = win_of(uni(knv));
        if (lane == 0) knv = atomicAdd(&s_next, 1u);
      }
      loaded = true;
      if (g >= b1) {
        mm.valid = false;
        mm.blk = 0;
        mm.p = base;
        mm.l = 0;
        return;
      }
      uint64_t gv = g;
      asm volatile("" : "+s"(gv));  // window address computed afresh each refill
      const uint64_t j = gv + lane;
      const bool in = lane < W && j < b1;  // the window's messages
      const uint64_t oj = in ? (offs ? offs[j] : j * stride) : 0;
      const uint32_t lj = in ? (lens ? lens[j] : ulen) : 0;
      // consume the loads inside the refill branch (their vmcnt(0) stays here)
      wo_lo = (uint32_t)oj;
      wo_hi = (uint32_t)(oj >> 32);
      wl = lj;
      asm volatile("" : "+v"(wo_lo), "+v"(wo_hi), "+v"(wl));
      // fast_mask != 0: the streaming kernel of this batch took the 16-B aligned
      // blocks whose length is a positive multiple of fast_mask + 1
      const bool fast = (((uintptr_t)base + oj) & 15u) == 0 && (lj & fast_mask) == 0 && lj != 0;
      todo = __ballot(in && !(fast_mask && fast));
      if constexpr (kSmallLanes) {
        if (msg) {
          const uint64_t sm = __ballot(in && !(fast_mask && fast) && lj <= kSmallMax);
          if (sm) {
            small_lanes(sm, oj, lj, gv);
            todo &= ~sm;
          }
        }
      }
    }
  };

  // ---- per-message geometry ------------------------------------------------
  // Payload M (block mode: bytes [4, len); message mode: all) is hashed as the
  // virtual message zeros(z) || W0 || M of `rows` 1 KiB rows, right-aligned so
  // the last row ends at the payload end.  Row r, lane l covers payload
  // offsets 1024r - z - 4 + 16l .. +15.
  struct Geo {
    const uint8_t *P;  // payload start
    uint32_t Lp, rows, z, q, rb;
    uintptr_t Abase;   // 16-B aligned start of row 0's chunks
    bool shortblk;     // block mode, len < 4: "invalid block data"
  };
  auto geo = [&](const Msg &mm) {
    Geo e;
    e.shortblk = !msg && mm.l < 4;
    e.P = msg ? mm.p : mm.p + 4;
    e.Lp = msg ? mm.l : (e.shortblk ? 0u : mm.l - 4);
    const uint64_t Lv = (uint64_t)e.Lp + 4;
    e.rows = (uint32_t)((Lv + kRowBytes - 1) / kRowBytes);
    e.z = (uint32_t)((uint64_t)e.rows * kRowBytes - Lv);
    const uintptr_t A0 = (uintptr_t)e.P - e.z - 4;
    const uint32_t m = (uint32_t)(A0 & 15u);
    e.q = m >> 2;
    e.rb = m & 3u;
    e.Abase = A0 - m;
    return e;
  };
  // Edge rows 0 and 1 (they may hold the virtual prefix; z + 4 <= 1027): each
  // lane loads the two aligned 16-B chunks around its window through a range
  // [P & ~15, roundup16(P + Lp)); chunks that do not overlap the payload get an
  // out-of-range offset, so no byte outside the payload's aligned chunks (its
  // own pages) is touched.  Also the stored word (block mode) through a 4-byte range.
  auto issue_edge = [&](const Msg &mm, const Geo &e, uint4 (&ch)[4], uint32_t &sw) {
    const uintptr_t P = (uintptr_t)e.P, Pa = P & ~(uintptr_t)15;
    const uint64_t span = mm.valid ? (((uint64_t)P + e.Lp + 15) & ~(uint64_t)15) - Pa : 0;
    const __amdgpu_buffer_rsrc_t re = buf_range((const void *)Pa, (uint32_t)(span < 0xFFFFFFF0ull ? span : 0xFFFFFFF0ull));
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uintptr_t X = e.Abase + (uintptr_t)r * kRowBytes + 16u * lane + 16u * h;
        const bool in = (uint32_t)r < e.rows && X + 16 > P && X < P + e.Lp;
        ch[2 * r + h] = buf_load16(re, in ? (uint32_t)(X - Pa) : 0xFFFFFFFFu);
      }
    const __amdgpu_buffer_rsrc_t rs = buf_range(mm.p, (mm.valid && !msg && !e.shortblk) ? 4u : 0u);
    sw = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, 0, 0, 0);
  };
  // Body rows >= 2 start inside the payload (2048 > z + 4): one unaligned 16-B
  // load per lane through the range [row 2, row `rows`); rows past the end are
  // out of range (zeros, no memory access).
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto issue_body = [&](const __amdgpu_buffer_rsrc_t rb_, uint32_t r0, u32x4 (&v)[kAnyBatch]) {
#pragma unroll
    for (int b = 0; b < kAnyBatch; b++) {
      const uint4 t = buf_load16(rb_, (r0 + b - 2) * kRowBytes + 16u * lane);
      v[b] = u32x4{t.x, t.y, t.z, t.w};
    }
  };
  auto hash_body = [&](const Geo &e, uint32_t r0, const u32x4 (&v)[kAnyBatch], uint32_t (&c)[4]) {
#pragma unroll
    for (int b = 0; b < kAnyBatch; b++)
      if (r0 + b < e.rows) {
        c[0] = row_step(c[0], v[b].x);
        c[1] = row_step(c[1], v[b].y);
        c[2] = row_step(c[2], v[b].z);
        c[3] = row_step(c[3], v[b].w);
      }
  };

  Msg cur;
  next(cur);
  if (!cur.valid) return;
  Geo ge = geo(cur);
  uint4 ch[4];
  uint32_t sw;
  auto body_range = [&](const Geo &e) {
    const uintptr_t A0 = e.Abase + e.q * 4 + e.rb;
    return buf_range((const void *)(A0 + 2 * kRowBytes), e.rows > 2 ? (e.rows - 2) * kRowBytes : 0u);
  };
  u32x4 VA[kAnyBatch];
  auto issue_first = [&](const Geo &e) {
    if (e.rows > 2) issue_body(body_range(e), 2, VA);
  };
  issue_edge(cur, ge, ch, sw);
  issue_first(ge);
  bool reported = false;  // wave-uniform: this wave already lowered first_bad (see k_crc_fast)
  for (;;) {
    const __amdgpu_buffer_rsrc_t rbody = body_range(ge);
    // edge rows
    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 2; r++) {
      if ((uint32_t)r < ge.rows) {
        const uint4 fw = funnel16(ch[2 * r], ch[2 * r + 1], ge.q, ge.rb);
        uint32_t w[4] = {fw.x, fw.y, fw.z, fw.w};
        const int64_t srow = (int64_t)r * kRowBytes - (int64_t)ge.z - 4;
        if (srow < 0) {  // zeros, then W0, then data
          // word k2 starts d bytes before the payload: keep its bytes j >= d,
          // and bytes ob = j - d in [-4, -1] are W0's byte ob + 4, i.e. the
          // window of Y = W0 << 32 that starts at byte 8 - d
          const uint64_t Y = (uint64_t)w0 << 32;
#pragma unroll
          for (int k2 = 0; k2 < 4; k2++) {
            const int32_t d = -((int32_t)srow + 16 * (int32_t)lane + 4 * k2);
            const uint32_t dm = d <= 0 ? 0xFFFFFFFFu : (d >= 4 ? 0u : 0xFFFFFFFFu << (8 * d));
            const uint32_t wv = (d >= 1 && d <= 8) ? (uint32_t)(Y >> (64 - 8 * d)) : 0u;
            w[k2] = (w[k2] & dm) | wv;
          }
        }
#pragma unroll
        for (int k2 = 0; k2 < 4; k2++) c[k2] = r == 0 ? w[k2] : row_step(c[k2], w[k2]);
      }
    }
    // every edge load is consumed here on every path (rows == 1 skips row 1's
    // hash), else the waitcnt pass assumes them pending at the loop headers
    // below and drains the queue there (vmcnt(0))
    asm volatile("" ::"v"(ch[0].x), "v"(ch[1].x), "v"(ch[2].x), "v"(ch[3].x), "v"(sw));
    const uint32_t dsw = uni(sw);
    // body rows, one batch at a time.  tools/kmsg measured this against a
    // double-buffered loop (the next batch in flight while one is hashed):
    // single batches were 4-12 % faster -- more bytes in flight per wave than
    // ~4 KiB do not help at 16 waves per CU (k_crc_fast: ring 4 beat ring 8)
    // (rolling refills in k_crc_grp's order -- row r+4 loaded right after row r
    // is hashed -- were 3-11 % slower: profiles/r2/any_rolling/)
    // (a double-buffered body -- the next batch in flight while one is hashed,
    // the batch past the end out of range, no branch -- was 7-10 % slower:
    // profiles/r2/any_double/)
    for (uint32_t r0 = 2; r0 < ge.rows; r0 += kAnyBatch) {
      if (r0 > 2) issue_body(rbody, r0, VA);
      hash_body(ge, r0, VA, c);
    }
    // the next message's edge rows go out before this one is finalised
    const Msg done = cur;
    const bool dshort = ge.shortblk;
    next(cur);
    ge = geo(cur);
    issue_edge(cur, ge, ch, sw);
    issue_first(ge);

    const uint32_t dd = shift4(shift4(shift4(c[0], c[1]), c[2]), c[3]);
    const uint32_t crcv = dshort ? 0u : wave_xor(matvec32(col, dd)) ^ 0xFFFFFFFFu;
    const bool bad = !msg && first_bad && (dshort || dsw != crcv);  // wave-uniform
    if (crc_out) lane0_store_u32(crc_out + done.blk, crcv);
    if (!msg && !dshort && (flags & kFlagStamp))  // PutUint32LE(block[0:4], crc)
      lane0_store_u32(reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(done.p)), crcv);
    if (bad) {
      if (bad_bitmap) lane0_atomic_or(bad_bitmap + (done.blk >> 5), 1u << (done.blk & 31));
      if (!reported) lane0_atomic_umin64(first_bad, done.blk);
      reported = true;
    }
    if (!cur.valid) return;
  }
}

template <bool kSmallLanes>
__global__ __launch_bounds__(kFastThreads) void k_crc_any(
    const uint8_t *base, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
    uint64_t stride, uint32_t ulen, uint32_t flags, uint64_t nblocks, uint32_t fast_mask, uint32_t lg_chunk,
    uint32_t *__restrict__ crc_out, uint32_t *__restrict__ bad_bitmap,
    unsigned long long *__restrict__ first_bad, const DeviceTables *__restrict__ tables,
    const unsigned long long *skip_slot = nullptr, uint64_t skip_tag = 0) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4 + 1];
  crc_any_body<kSmallLanes>(lds, base, offs, lens, stride, ulen, flags, nblocks, fast_mask, lg_chunk, crc_out,
                            bad_bitmap, first_bad, tables, skip_slot, skip_tag);
}

// ---------------------------------------------------------------------------
// Edge blocks of AddCRCsToData framing (the first, whose row 0 would start 4
// bytes before src, and the last, whose payload may end mid-row): aligned
// loads predicated on the payload range + funnel shift + byte masks -- never
// touches a byte outside src.  Stores block b's rows (lane 0's first 16 bytes
// are returned in `keep` for the caller to store with the CRC in front) and
// leaves the four Horner streams in c (lane 0's row-0 word 0 = W0).
template <class RowStep>
__device__ __forceinline__ void frame_edge_rows(uint64_t b, const uint8_t *__restrict__ src, uint64_t n,
                                                uint8_t *__restrict__ dst, uint32_t lane, uint32_t w0,
                                                RowStep row_step, uint32_t (&c)[4], uint4 &keep) {
  constexpr uint64_t kPay = 4092;  // BLOCK_SIZE - CRC_SIZE (crc_util.go:43)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const uintptr_t P = (uintptr_t)src + b * kPay;                      // payload start
  const uint64_t len = (n - b * kPay) < kPay ? (n - b * kPay) : kPay;  // payload bytes
  const uintptr_t S0 = P - 4;                                          // source of output byte 0
  const uint32_t m = (uint32_t)(S0 & 15u), q = m >> 2, rb = m & 3u;
  const uintptr_t Ab = S0 - m;
  uint4 ch0[4], ch1[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uintptr_t X0 = Ab + (uintptr_t)r * kRowBytes + 16u * lane, X1 = X0 + 16;
    ch0[r] = ch1[r] = make_uint4(0, 0, 0, 0);
    if (X0 + 16 > P && X0 < P + len) ch0[r] = load_row(reinterpret_cast<const uint8_t *>(X0), 0);
    if (X1 + 16 > P && X1 < P + len) ch1[r] = load_row(reinterpret_cast<const uint8_t *>(X1), 0);
  }
  keep = make_uint4(0, 0, 0, 0);
  uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint4 fw = funnel16(ch0[r], ch1[r], q, rb);
    uint32_t w[4] = {fw.x, fw.y, fw.z, fw.w};
    // keep output bytes t (= 1024r + 16l + 4k + j) with 4 <= t < 4 + len
    const int32_t hi = 4 + (int32_t)len - (r * (int32_t)kRowBytes + 16 * (int32_t)lane);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t nb = hi - 4 * k;  // bytes of this word still inside the payload
      uint32_t dm = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
      if (r == 0 && k == 0) dm &= lane == 0 ? 0u : 0xFFFFFFFFu;  // bytes 0..3: the CRC field
      w[k] &= dm;
    }
    const u32x4 outv = {w[0], w[1], w[2], w[3]};
    if (r == 0 && lane == 0) {
      keep = make_uint4(w[0], w[1], w[2], w[3]);
      w[0] = w0;  // Go's init in place of the CRC field
    } else {
      __builtin_nontemporal_store(outv, reinterpret_cast<u32x4 *>(ob + r * kRowBytes + 16 * lane));
    }
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : row_step(c[k], w[k]);
  }
}

// ---------------------------------------------------------------------------
// The row step without LDS (k_unframe): a 32x32 GF(2) mat-vec M.c is the XOR
// of five 64-entry tables T_j[6-bit chunk j of c] (bits 0..29) and the two
// columns of bits 30, 31.  Each table sits in ONE VGPR -- lane v holds T_j[v]
// -- and is read by ds_bpermute_b32, the cross-lane gather: no LDS allocation,
// no bank conflicts, no table fill, so a kernel built on it can run as
// short-lived 4-wave workgroups.  The columns come from the
// constant image: column i of shift(., 1024) is tg[i/8][1 << i%8], of
// shift(., 4) s4[i/8][1 << i%8].  ds_bpermute reads only address bits 7..2,
// so the chunk addresses need no mask.
struct XTab {
  uint32_t t[5];
  uint32_t c30, c31;  // wave-uniform
};
__device__ __forceinline__ XTab make_xtab(const uint32_t (*tab)[256], uint32_t lane) {
  XTab r;
#pragma unroll
  for (int j = 0; j < 5; j++) {
    uint32_t e = 0;
#pragma unroll
    for (int b = 0; b < 6; b++) {
      const int i = 6 * j + b;
      const uint32_t m = 0u - ((lane >> b) & 1u);
      e = __builtin_amdgcn_bitop3_b32(m, tab[i >> 3][1u << (i & 7)], e, 0x6A);  // (m & col) ^ e
    }
    r.t[j] = e;
  }
  r.c30 = tab[3][1u << 6];
  r.c31 = tab[3][1u << 7];
  return r;
}
// M.c ^ w
__device__ __forceinline__ uint32_t xapply(const XTab &T, uint32_t c, uint32_t w) {
  uint32_t g[5];
#pragma unroll
  for (int j = 0; j < 5; j++)
    g[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j == 0 ? (c << 2) : (c >> (6 * j - 2))), (int)T.t[j]);
  const uint32_t m30 = (uint32_t)((int32_t)(c << 1) >> 31), m31 = (uint32_t)((int32_t)c >> 31);
  uint32_t a = __builtin_amdgcn_bitop3_b32(m30, T.c30, w, 0x6A);
  a = __builtin_amdgcn_bitop3_b32(m31, T.c31, a, 0x6A);
  return xor3(xor3(g[0], g[1], g[2]), g[3], xor3(g[4], a, 0u));
}

// The lane placement's 32 columns shared by a 4-wave workgroup: one 8 KiB LDS
// copy of DeviceTables::lane_q (every load issued before the first store), read
// back with 8 ds_read_b128 per placement (lane l's 16 B of each quarter are
// consecutive: no bank conflicts).  Loading the 128 B of columns per lane from
// L2 instead (8 KiB per wave) held the framing kernels at one block per wave
// to 4.56 TB/s; shared, one block per wave is the fastest geometry
// (tools/kframe3, profiles/r3/framing_lq/).
__device__ __forceinline__ void fill_lane_q(uint32_t *lq, const DeviceTables *__restrict__ tables) {
  constexpr uint32_t kQ = kLaneQWords / 4, kPer = kQ / 256;  // uint4s; per thread of 256
  static_assert(kQ % 256 == 0, "lane_q copy: whole uint4s per thread");
  const uint4 *g = reinterpret_cast<const uint4 *>(&tables->lane_q[0][0][0]);
  uint4 t[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) t[k] = g[threadIdx.x + k * 256u];
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[threadIdx.x + k * 256u] = t[k];
}
// the 32x32 mat-vec of lane `lane`'s placement matrix with d (matvec32 against LDS columns)
__device__ __forceinline__ uint32_t place_lq(const uint32_t *lq, uint32_t lane, uint32_t d) {
  uint32_t acc = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint4 c4 = reinterpret_cast<const uint4 *>(lq)[q * kLanes + lane];
    const uint32_t cq[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t m = (uint32_t)((int32_t)(d << (31 - (4 * q + r))) >> 31);  // bit 4q+r of d, spread
      acc = __builtin_amdgcn_bitop3_b32(m, cq[r], acc, 0x6A);                   // (m & col) ^ acc
    }
  }
  return acc;
}

// XCD-contiguous workgroup order for the short-lived framing kernels:
// workgroup i is dispatched to XCD i % 8, so it takes logical workgroup
// (i % 8) * (G8 / 8) + i / 8 (G8 = G rounded down to a multiple of 8; the last
// G % 8 keep their index).  Each XCD's L2 then sees one contiguous stretch of
// blocks, and the 128-B lines that neighbouring blocks share (4092-B payload
// strides) meet in one L2 instead of two: +4.6-5 % for k_frame and k_unframe
// (tools/kframe4 KF4_SET=xcd, profiles/r3/kframe4/).
__device__ __forceinline__ uint32_t xcd_wg(uint32_t i, uint32_t G) {
  const uint32_t G8 = G & ~7u;
  return i < G8 ? (i & 7u) * (G8 >> 3) + (i >> 3) : i;
}

// ---------------------------------------------------------------------------
// Fused AddCRCsToData (utils/crc/crc_util.go:41-64, row f2): payload slices of
// 4092 B -> 4096-B blocks with the CRC in front, one read of the payload and
// one write of the blocks.  One launch of k_frame (launch_frame):
//   workgroup 0    the first block (row 0 would start 4 bytes before src) and
//                  the last (ragged payload): aligned, range-predicated loads,
//                  funnel shift and byte masks, one wave each -- no byte
//                  outside src is touched (frame_edges_wave).
//   the others     interior blocks 1 .. nblk-2: every row window lies inside
//                  src, so each lane's 16 output bytes come from two aligned
//                  16-B chunks (its own and its neighbour's, by DPP) without
//                  masks.  One block per wave, 4-wave workgroups that exit:
//                  row steps and the stream combine through XTab (no LDS
//                  tables to fill), the lane placement against the
//                  workgroup's LDS copy of its columns.  Rows 1-3 are stored
//                  before the hash (the other orders within +-0.5 %), row 0
//                  after it with the CRC in front (one write of the line).
// Round 2's kernel (persistent 16-wave workgroups, 144 KiB of LDS tables)
// ran 5.10-5.24 TB/s; this one 5.26-5.48 on the same boxes (tools/kframe3).
// The first block (row 0 would start 4 bytes before src) and the last (ragged
// payload), by waves 0 and 1 of k_frame's workgroup 0 (the workgroup's columns
// in LDS already; waves 2 and 3 only help fill them).  Aligned,
// range-predicated loads, funnel shift and byte masks: no byte outside src is
// touched.  Until late round 3 this was its own launch (k_frame_edges, ~5 us
// plus the gap between the two kernels, ~0.4 % of a 1M-block call).
__device__ __forceinline__ void frame_edges_wave(const uint8_t *__restrict__ src, uint64_t n,
                                                 uint8_t *__restrict__ dst, uint64_t nblk,
                                                 uint32_t *__restrict__ crc_out, const uint32_t *lq,
                                                 const XTab &TM, const XTab &TS, uint32_t w0, uint32_t lane,
                                                 uint32_t wv) {
  const uint64_t b = wv == 0 ? 0 : nblk - 1;
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t { return xapply(TM, c, w); };
  uint32_t c[4];
  uint4 keep;
  frame_edge_rows(b, src, n, dst, lane, w0, row_step, c, keep);
  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;
  if (lane == 0) {
    keep.x = crcv;  // binary.LittleEndian.PutUint32(block[:4], crc)
    *reinterpret_cast<uint4 *>(dst + b * (uint64_t)HC_FRAME_BLOCK) = keep;
    if (crc_out) crc_out[b] = crcv;
  }
}

__global__ __launch_bounds__(256) void k_frame(const uint8_t *__restrict__ src, uint64_t n, uint8_t *__restrict__ dst,
                                               uint64_t nblk, uint32_t *__restrict__ crc_out,
                                               const DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr uint64_t kPay = 4092;  // BLOCK_SIZE - CRC_SIZE (crc_util.go:43)
  __shared__ __attribute__((aligned(16))) uint32_t lq[kLaneQWords];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wg = xcd_wg(blockIdx.x, gridDim.x);  // logical workgroup (workgroup 0 stays 0)
  if (wg == 0) {  // the edge blocks first (dispatched early, overlapped with the interior)
    fill_lane_q(lq, tables);
    const uint32_t wv = uni(threadIdx.x >> 6);
    const XTab TM = make_xtab(tables->tg, lane);
    const XTab TS = make_xtab(tables->s4, lane);
    __syncthreads();
    if (wv == 0 || (wv == 1 && nblk >= 2)) frame_edges_wave(src, n, dst, nblk, crc_out, lq, TM, TS, tables->w0, lane, wv);
    return;
  }
  // interior logical workgroup I = wg - 1 takes interior blocks S (4 (I / S) +
  // w) + I % S (S = kFrameSpread = 8): b mod 4 fixes the source's misalignment
  // (4092 b mod 16), so a workgroup's four waves share it and read no shared
  // line (+3.8 % with S = 4, +1.2 % more with S = 8; profiles/r3/kframe4/); the
  // interior grid is a multiple of S workgroups (launch_frame)
  const uint32_t I = wg - 1;
  const uint64_t b = 1 + 4ull * kFrameSpread * (I / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + I % kFrameSpread;
  const bool mine = b + 1 < nblk;
  // A wave past the last interior block loads block 1's rows (interior
  // whenever this kernel runs) and exits after the barrier: no branch around
  // the row loads, so the waitcnt pass sees them on one path.
  const uint64_t bl = mine ? b : 1;
  // Aligned source loads: lane l's 16 output bytes of row r are bytes m .. m+15
  // of its aligned chunk C_l and the next one, C_{l+1}, which the right
  // neighbour loaded (a whole-wave DPP shift, wave_shl:1).  Lane 63's C_{l+1}
  // is lane 0's chunk of the next row (v_readlane, no memory access); only row
  // 3's, the chunk after the block, is loaded, through a buffer range in which
  // every other lane's offset is out of range (no branch around the load).
  // m = (S mod 16) is the block's misalignment, uniform over its rows.  Aligned
  // loads ran +3.5-4 % over one unaligned 16-B load per lane (tools/kframe3
  // KF3_SET=a); the one tail load instead of four, +2.6-3.1 % (tools/kframe4).
  const uintptr_t S = (uintptr_t)src + bl * kPay - 4;  // source of output byte 0
  const uint32_t m = (uint32_t)(S & 15u), qs = m >> 2, rs = m & 3u;
  const uintptr_t Sa = S - m;
  // [Sa, Sa + 4112) clipped to the aligned chunk holding src's last byte: the
  // buffer range check is per load, so the range ends on a 16-B boundary (as
  // k_crc_any's edge rows: no byte outside src's own aligned chunks is read)
  const uintptr_t end16 = ((uintptr_t)src + n + 15) & ~(uintptr_t)15;
  const __amdgpu_buffer_rsrc_t r63 =
      buf_range(reinterpret_cast<const void *>(Sa), (uint32_t)(end16 - Sa < 4112u ? end16 - Sa : 4112u));
  // The workgroup's placement columns (L2 hits) are loaded first, then the rows
  // (+0.6 % over the other order, tools/kframe4).  The row addresses are
  // integers, so the row loads are flat loads: global ones (src's provenance)
  // ran 1.5 % slower here.
  static_assert(kLaneQWords / 4 / 256 == 2, "two uint4s of columns per thread");
  const uint4 *lqg = reinterpret_cast<const uint4 *>(&tables->lane_q[0][0][0]);
  const uint4 lq0 = lqg[threadIdx.x], lq1 = lqg[threadIdx.x + 256u];  // named: an array was promoted to LDS
  __builtin_amdgcn_sched_barrier(0);
  u32x4 C[4];
#pragma unroll
  for (int r = 0; r < 4; r++)
    C[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Sa + r * kRowBytes + 16u * lane));
  const uint4 X3 = buf_load16(r63, lane == 63 ? 4096u : 0xFFFFFFFFu);
  __builtin_amdgcn_sched_barrier(0);
  reinterpret_cast<uint4 *>(lq)[threadIdx.x] = lq0;
  reinterpret_cast<uint4 *>(lq)[threadIdx.x + 256u] = lq1;
  const XTab TM = make_xtab(tables->tg, lane);
  const XTab TS = make_xtab(tables->s4, lane);
  const uint32_t w0 = tables->w0;
  __syncthreads();
  if (!mine) return;
  auto wave_shl1 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false); };
  auto lane0_of = [](const u32x4 x) {  // lane 0's chunk, wave-uniform
    return make_uint4(__builtin_amdgcn_readlane(x.x, 0), __builtin_amdgcn_readlane(x.y, 0),
                      __builtin_amdgcn_readlane(x.z, 0), __builtin_amdgcn_readlane(x.w, 0));
  };
  u32x4 v[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint4 a = make_uint4(C[r].x, C[r].y, C[r].z, C[r].w);
    uint4 nb = make_uint4(wave_shl1(a.x), wave_shl1(a.y), wave_shl1(a.z), wave_shl1(a.w));
    const uint4 t = r < 3 ? lane0_of(C[r < 3 ? r + 1 : 3]) : X3;
    if (lane == 63) nb = t;
    const uint4 f = funnel16(a, nb, qs, rs);
    v[r] = u32x4{f.x, f.y, f.z, f.w};
  }
  uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
  // Rows 1-3 now; row 0 after the hash, with the CRC in lane 0's word: one
  // store of the block's first line, not a zero word now and a 4-byte CRC store
  // later, which left the L2 as a partial write (0.77M partial 32-B write
  // requests per 1M blocks, profiles/r4/r4jj/; +0.9 %, r4kk/ab_frame/)
#pragma unroll
  for (int r = 1; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4 *>(ob + r * kRowBytes));
  uint32_t c[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    u32x4 t = v[r];
    if (r == 0) t.x = lane == 0 ? w0 : t.x;  // Go's init in place of the CRC field
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : xapply(TM, c[k], w[k]);
  }
  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;
  u32x4 t0 = v[0];
  t0.x = lane == 0 ? crcv : t0.x;  // lane 0's ob is the block start
  __builtin_nontemporal_store(t0, reinterpret_cast<u32x4 *>(ob));
  if (crc_out) lane0_store_u32(crc_out + b, crcv);
}

// ---------------------------------------------------------------------------
// Batched ReadFromDisk on device (lsm/block_manager/block_manager.go:203-235,
// row f1): verify every block of a contiguous run (CheckBlockIntegrity,
// crc_util.go:88-100) and strip the CRC words, writing the payloads back to
// back (block b's block[4:B] at out + b*(B-4)) -- the inverse of k_frame, one
// read of the blocks and one write of the payload.  B = 4096 << lg_groups.
//   * 4-wave workgroups, each wave one 4 KiB block, or one 4 KiB group of an
//     8/16 KiB block (the block's groups combined through LDS, below), then
//     exit.  The persistent 16-wave version with 144 KiB of LDS tables ran 5.0-5.2
//     TB/s; four blocks per wave with the placement columns loaded per lane
//     5.45-5.62; one block per wave with them shared in LDS 6.04
//     (tools/kframe3, profiles/r3/framing/, profiles/r3/framing_lq/).
//   * Row steps and the stream combine through XTab (ds_bpermute); the lane
//     placement is the 32x32 mat-vec against the workgroup's LDS copy of its
//     columns (place_lq).
//   * Payload stores are 16-B unaligned stores (output is shifted 4 bytes per
//     block).  The block's first 12 payload bytes: at 4 KiB a 12-B store by
//     lane 0; at 8/16 KiB lane 0 of group 0 stores bytes 4..19 (lane 1's first
//     word via DPP), overlapping lane 1's store with identical bytes.
//     A group's four rows are hashed, then its four stores are issued together
//     (+3.9 % over storing each row before hashing it, profiles/r2/framing_store/).
//   * first_bad: a wave lowers it at most once, and only after reading it
//     (a batch of all-bad blocks would otherwise put ~nblk/4 atomics on one word).
template <uint32_t lg_groups>
__global__ __launch_bounds__(256) void k_unframe(const uint8_t *blocks, uint64_t nblk,  // (not restrict: below)
                                                 uint8_t *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                 uint32_t *__restrict__ bad_bitmap,
                                                 unsigned long long *__restrict__ first_bad,
                                                 const DeviceTables *__restrict__ tables) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint32_t kGroups = 1u << lg_groups, gmask = kGroups - 1u;
  constexpr uint64_t B = (uint64_t)HC_FRAME_BLOCK << lg_groups, Bp = B - 4;
  __shared__ __attribute__((aligned(16))) uint32_t lq[kLaneQWords];
  const uint32_t lane = threadIdx.x & 63;
  if constexpr (lg_groups == 0) {
    // 4 KiB blocks, one a wave: straight-line code with a wave-uniform block
    // index.  The group loop below, with the index taken from threadIdx as a
    // VGPR (exec-masked branches), ran 6.5 % slower (tools/kframe4: 5490 vs
    // 5830-5850 GB/s).  `blocks` is not __restrict__: with it, hipcc may sink
    // the row loads past the barrier into the block that uses them.
    // Logical workgroup L (XCD-contiguous) takes blocks S (4 (L / S) + w) + L % S
    // (S = kFrameSpread = 8): b mod 4 fixes the output's misalignment (4092 b
    // mod 16), so the four waves of a workgroup store with one alignment, and
    // no two of them write a shared line (+3.5 % with S = 4 over four
    // consecutive blocks, +2.6 % more with S = 8; profiles/r3/kframe4/); the
    // grid is a multiple of S workgroups (unframe_grid).
    const uint32_t L = xcd_wg(blockIdx.x, gridDim.x);
    const uint64_t b = 4ull * kFrameSpread * (L / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + L % kFrameSpread;
    const bool mine = b < nblk;
    const uint32_t w0 = tables->w0;
    u32x4 v[4];
    if (mine) {  // the rows before the table work
      const uint8_t *S = blocks + b * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
      for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * kRowBytes));
    }
    fill_lane_q(lq, tables);
    const XTab TM = make_xtab(tables->tg, lane);
    const XTab TS = make_xtab(tables->s4, lane);
    __syncthreads();
    if (!mine) return;
    uint32_t c[4] = {0, 0, 0, 0};
    uint32_t stored = 0;
    uint8_t *ob = out + b * Bp + 16u * lane - 4;
    u32x4 sv[4];
    uint8_t *sa[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      if (r == 0) {
        stored = __builtin_amdgcn_readfirstlane(t.x);  // LE32(block[0:4])
        sv[r] = t;
        sa[r] = ob;
        t.x = lane == 0 ? w0 : t.x;  // Go's init in place of the CRC field
      } else {
        sv[r] = t;
        sa[r] = ob + r * kRowBytes;
      }
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : xapply(TM, c[k], w[k]);
    }
    // Lane 0's row-0 bytes 4..15 (the block's first 12 payload bytes) go out by
    // a 12-B store; the row-0 16-B store runs through a buffer range in which
    // lane 0 is out of range.  Round 3's form (lane 0 storing bytes 4..19, four
    // of them over lane 1's) ran 76.3 against 77.9 % (profiles/r4/r4pp/ab_unf/);
    // the same change at 8/16 KiB (group 0's head) lost 1 point (ab_unf8/16).
    {
      typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
      const __amdgpu_buffer_rsrc_t r0 = buf_range(out + b * Bp - 4, kRowBytes);
      __builtin_amdgcn_raw_buffer_store_b128(sv[0], r0, lane == 0 ? 2u * kRowBytes : 16u * lane, 0, 2);
      const __amdgpu_buffer_rsrc_t rh = buf_range(out + b * Bp, 12u);
      __builtin_amdgcn_raw_buffer_store_b96(u32x3{sv[0].y, sv[0].z, sv[0].w}, rh, lane == 0 ? 0u : 16u, 0, 2);
    }
#pragma unroll
    for (int r = 1; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
    const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
    const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;
    if (crc_out) lane0_store_u32(crc_out + b, crcv);
    if (first_bad && crcv != stored) {  // wave-uniform; one block a wave: at most one lowering
      if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
      if (b < __hip_atomic_load(first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) lane0_atomic_umin64(first_bad, b);
    }
  } else {
    // 8/16 KiB blocks: one 4 KiB group per wave, a block's 2 or 4 groups in
    // one workgroup.  Each wave hashes and stores its group exactly as a 4 KiB
    // block (the group's raw CRC register r_g, zero init unless g = 0), shifts
    // r_g past the groups after it (4096 * (G-1-g) bytes: a 32x32 mat-vec on a
    // wave-uniform value, one column per lane, DeviceTables::sh4k), and the
    // last group's wave XORs the block's r_g from LDS and reports.  One wave
    // per block with the groups in turn (each group's rows prefetched during
    // the previous one) ran 5.17-5.34 TB/s; every wave with one group's rows
    // in flight is the 4 KiB kernel's pattern.
    __shared__ uint32_t reg[4], st_word[4];
    const uint32_t wave = uni(threadIdx.x >> 6);
    const uint32_t L = xcd_wg(blockIdx.x, gridDim.x);
    // 16 KiB: one block per workgroup.  8 KiB: workgroup L takes blocks
    // 8 (L / 4) + L % 4 and that + 4 (waves 0-1 and 2-3), which share b mod 4
    // and so one output alignment (as the 4 KiB path; unframe_grid covers whole
    // groups of 8 blocks)
    const uint64_t b = lg_groups == 1 ? 8ull * (L >> 2) + (L & 3u) + 4u * (wave >> 1)
                                      : ((uint64_t)L * 4 + wave) >> lg_groups;
    const uint32_t g = wave & gmask;
    const bool mine = b < nblk;
    const uint32_t w0 = tables->w0;
    u32x4 v[4];
    if (mine) {
      const uint8_t *S = blocks + b * B + (uint64_t)g * HC_FRAME_BLOCK + 16u * lane;
#pragma unroll
      for (int r = 0; r < 4; r++) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(S + r * kRowBytes));
    }
    fill_lane_q(lq, tables);
    const XTab TM = make_xtab(tables->tg, lane);
    const XTab TS = make_xtab(tables->s4, lane);
    const uint32_t shcol = g < gmask ? tables->sh4k[gmask - 1u - g][lane & 31u] : 0u;
    __syncthreads();
    if (!mine) return;  // (ended waves do not hold up the barrier below)
    uint32_t c[4] = {0, 0, 0, 0};
    uint8_t *ob = out + b * Bp + (uint64_t)g * HC_FRAME_BLOCK + 16u * lane - 4;
    const bool head = g == 0 && lane == 0;  // the block's first 16 bytes: CRC field + 12 payload bytes
    u32x4 sv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      sv[r] = t;
      if (r == 0) {  // (selects, not branches: one store address form, a global store)
        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);  // lane+1's x
        if (head) st_word[wave >> lg_groups] = t.x;                                           // LE32(block[0:4])
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = head ? first : t;
        t.x = head ? w0 : t.x;  // Go's init in place of the CRC field
      }
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = r == 0 ? w[k] : xapply(TM, c[k], w[k]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
      __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(ob + r * kRowBytes + (r == 0 && head ? 4 : 0)));
    const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);
    uint32_t rg = wave_xor(place_lq(lq, lane, d));
    if (g < gmask) rg = wave_xor(lane < 32 && ((rg >> lane) & 1u) ? shcol : 0u);  // shift(r_g, 4096 (G-1-g))
    if (lane == 0) reg[wave] = rg;
    __syncthreads();
    if (g != gmask) return;
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kGroups; k++) tot ^= reg[wave - gmask + k];
    const uint32_t crcv = tot ^ 0xFFFFFFFFu;
    const uint32_t stored = st_word[wave >> lg_groups];
    if (crc_out) lane0_store_u32(crc_out + b, crcv);
    if (first_bad && crcv != stored) {  // one block a wave: at most one lowering
      if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
      if (b < __hip_atomic_load(first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) lane0_atomic_umin64(first_bad, b);
    }
  }
}

// ---------------------------------------------------------------------------
// Synthetic workload fill: 64-bit word w of block i = splitmix64(seed, i, w).
__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t blk, uint64_t w) {
  uint64_t z = seed + ((blk << 21) + w) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Block blk of the buffer is block first + blk of the synthetic batch (a rank's
// shard of a global batch holds exactly the bytes the whole batch has there).
__global__ __launch_bounds__(256) void k_fill(uint8_t *base, const uint64_t *off, const uint32_t *len,
                                               uint64_t stride, uint32_t ulen, uint64_t n,
                                               uint64_t seed, uint64_t first) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t W = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + uni(threadIdx.x >> 6); i < n; i += W) {
    const uint64_t o = off ? off[i] : i * stride;
    const uint32_t l = len ? len[i] : ulen;
    const uint64_t blk = first + i;
    uint8_t *p = base + o;
    if ((((uintptr_t)p) & 15u) == 0) {
      for (uint32_t w = 2 * lane; 8 * w + 16 <= l; w += 128) {
        ulonglong2 v;
        v.x = splitmix(seed, blk, w);
        v.y = splitmix(seed, blk, w + 1);
        *reinterpret_cast<ulonglong2 *>(p + 8 * w) = v;
      }
      // tail (l % 16 != 0)
      const uint32_t done = l & ~15u;
      for (uint32_t b = done + lane; b < l; b += 64)
        p[b] = (uint8_t)(splitmix(seed, blk, b >> 3) >> (8 * (b & 7)));
    } else {
      for (uint32_t b = lane; b < l; b += 64)
        p[b] = (uint8_t)(splitmix(seed, blk, b >> 3) >> (8 * (b & 7)));
    }
  }
}

__global__ void k_verify_prepare(uint32_t *bitmap, unsigned long long *first_bad, uint64_t words) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (bitmap)
    for (uint64_t k = i; k < words; k += (uint64_t)gridDim.x * blockDim.x) bitmap[k] = 0;
  if (i == 0 && first_bad) *first_bad = (unsigned long long)LLONG_MAX;
}

// ---------------------------------------------------------------------------
// Packed whole-message batches (records back to back: off[i+1] = off[i] +
// len[i], GetCRC of each; config 5's per-record variant) by ONE stream over
// their span instead of one wave per record.  raw is linear, so every record
// [a, b) is ChecksumIEEE = raw(a .. b) ^ shift(~0, b - a) ^ ~0 with raw(a .. b)
// from the span's raw CRCs at a and b relative to any common origin; the stream
// only has to leave them at the record boundaries ("events"), relative to the
// 16 KiB unit holding each event.
//   k_seg_plan     events -> first event of every 16 KiB unit; per workgroup,
//                  which modes its records rule out, their gap bytes against
//                  their payload, and how many are k_crc_grp's blocks (slots
//                  that k_seg_stream's prologue reduces to the mode word)
//   k_seg_stream   k_crc_grp's rows, groups and hand-out over the span's units;
//                  per unit its raw CRC, and at every row holding events
//                  H(x) = shift(raw(unit .. x), re - x) (re = the row's end):
//                  the row start's value from the Horner streams, the row's
//                  bytes before x placed at the row end (lane placement of the
//                  whole lane chunks before x by an exclusive XOR scan, of the
//                  event's own lane chunk masked at x)
//   k_seg_combine  per record: H(a) and H(b) plus the raw CRCs of the whole
//                  units between them, advanced to re_b, then one inverse
//                  shift by re_b - b (SegTables: 6 table multiplies a record).
constexpr uint32_t kSegUnitLg = 14;  // unit = 16 KiB = 16 rows = 4 groups (the kernels take it as kU)
constexpr uint32_t kSegMaxRecord = 1u << 24;  // longest record the stream takes (16 MiB)
constexpr uint64_t kSegMaxGap = 1u << 22;     // longest gap between two records it takes (4 MiB)
constexpr uint64_t kSegSmallGap = 64;         // longest gap k_seg_combine hashes itself (kSegGapSmall)
constexpr uint32_t kSegPlanMaxWgs = 16384;   // k_seg_plan's largest grid: one "bad" slot per workgroup
constexpr uint32_t kSegPlanWgs = 2048;       // its default grid cap (grid-stride beyond; r4e: 13.5 vs 16.8 us at 2M events)
constexpr uint32_t kSegSyncGroups = 16;      // the sort's barrier tree: group counters (seg_sync)

struct SegGeo {
  uint64_t a0, pend, units;
};
template <uint32_t kU = kSegUnitLg>
__device__ __forceinline__ SegGeo seg_geo(const uint8_t *base, const uint64_t *offs, const uint32_t *lens,
                                          uint64_t n) {
  SegGeo g;
  g.a0 = ((uint64_t)base + offs[0]) & ~1023ull;
  g.pend = (uint64_t)base + offs[n - 1] + lens[n - 1];
  g.units = ((g.pend - g.a0) >> kU) + 1;
  return g;
}

// Two event lists, one plan.  A packed batch (off[j] = off[j-1] + len[j-1])
// has the n + 1 events s_0 .. s_{n-1}, pend (record j = events j, j+1).  A
// sorted batch with gaps (round 5: off[j] >= off[j-1] + len[j-1], e.g. WAL
// records behind their 17-B headers) has the 2n events s_0, e_0, s_1, e_1, ..
// (record j = events 2j, 2j+1; e_{n-1} = pend); the identity of the stream
// (raw(a .. b) from G(a) and G(b)) does not need the records to touch.
// first_ev[u] = the first event at or after unit u's start, in the gapped
// numbering (u = 0 .. units; first_ev[units] = 2n + 2); for a packed batch
// e_{j-1} and s_j coincide, so its packed number is (first_ev[u] + 1) >> 1.
// Workgroup w writes plan_bad[w]: bit 0 when its records find the batch not
// packed or with more than 64 packed events in one 4 KiB group (records under
// ~64 B), bit 1 when they find records out of order or overlapping, a gap over
// kSegMaxGap, or more than 64 gapped events in a group; both when the span exceeds max_units, a
// record exceeds kSegMaxRecord or lies outside [s_0, pend].  plan_gx[w] =
// sum over its records of 4 * (gap before it) - len: the stream takes a gapped
// batch only when the grid's sum is <= 0 (gap bytes at most a quarter of the
// payload, the span-DMA rule of the host pipeline).  Every slot is written, so
// the dispatch needs no memset: k_seg_stream's workgroups reduce the slots and
// its workgroup 0 stores the mode the combine reads.
// The plan of one batch over workgroup wg of nwg (blockDim.x threads each),
// with the workgroup's shared words: k_seg_plan's body, and the plan of the
// sorted view inside k_seg_stream (seg_sort).
struct SegPlanShared {
  uint32_t bad, conf;
  unsigned long long gx;
};
template <uint32_t kU>
__device__ __forceinline__ void seg_plan_body(const uint8_t *base, const uint64_t *__restrict__ offs,
                                              const uint32_t *__restrict__ lens, uint64_t n, uint64_t max_units,
                                              uint32_t wg, uint32_t nwg, uint32_t *__restrict__ plan_bad,
                                              long long *__restrict__ plan_gx, uint32_t *__restrict__ plan_conf,
                                              uint32_t *__restrict__ first_ev, SegPlanShared &sh) {
  if (threadIdx.x == 0) {
    sh.bad = 0;
    sh.conf = 0;
    sh.gx = 0;
  }
  const uint64_t step = (uint64_t)nwg * blockDim.x;
  // records k_crc_grp would take (the fallback's choice: k_seg_stream
  // prologue), counted in the checking loop below and, past a thread's early
  // stop, in a loop of their own (round 5 counted them in a first pass over
  // the arrays: one more dependent round trip per record a thread)
  uint32_t conf = 0;
  auto grp_rec = [&](uint64_t s, uint32_t l) -> uint32_t { return (s & 15u) == 0 && l && (l & 4095u) == 0 ? 1u : 0u; };
  const SegGeo g = seg_geo<kU>(base, offs, lens, n);
  uint32_t bad = g.units > max_units || n >= 0x7FFFFFFFull || g.pend < g.a0 ? 15u : 0u;
  const uint64_t s0 = (uint64_t)base + offs[0];
  long long gx = 0;
  auto grp = [&](uint64_t p) { return (p - g.a0) >> 12; };
  // bits: 1 not packed (or a packed group of 65 events), 2 not the zeroed-gap
  // mode (out of order, overlapping, a gap over kSegMaxGap, 65 of the 2n
  // events in a group), 4 a gap over kSegSmallGap, 8 not the small-gap mode
  // (out of order, overlapping, 65 of its n + 1 events -- record ends -- in a
  // group).  A thread stops when no mode is left.
  auto none_left = [](uint32_t b) { return (b & 1u) && (b & 2u) && (b & 12u); };
  uint64_t j = (uint64_t)wg * blockDim.x + threadIdx.x;
  for (; j < n && !none_left(bad); j += step) {
    const uint64_t s = (uint64_t)base + offs[j], l = lens[j], e = s + l;
    conf += grp_rec(s, (uint32_t)l);
    if (l > kSegMaxRecord || s < g.a0 || e > g.pend) {  // k_seg_combine's unit chain stays <= 1025 units
      bad = 15u;
      j += step;
      break;
    }
    uint64_t ulo = 0;
    if (j > 0) {
      const uint64_t sp = (uint64_t)base + offs[j - 1], ep = sp + lens[j - 1];
      if (s != ep) bad |= 1u;
      // a gap over kSegMaxGap also refuses the gapped mode: first_ev is filled
      // by each record for the units back to its predecessor's end, which a
      // batch out of order would otherwise make O(n x units) writes (1M
      // shuffled 4 KiB records: 33 ms, profiles/r5/r5e/)
      if (s < ep || s - ep > kSegMaxGap) bad |= 2u;
      if (s < ep) bad |= 8u;
      if (s > ep + kSegSmallGap) bad |= 4u;
      gx += 4 * (long long)(s >= ep ? s - ep : 0);
      ulo = ((ep - g.a0) >> kU) + 1;
    }
    gx -= (long long)l;
    if (j >= 64 && grp(s) == grp((uint64_t)base + offs[j - 64])) bad |= 1u;
    if (j + 1 == n && n >= 64 && grp(g.pend) == grp((uint64_t)base + offs[n - 64])) bad |= 1u;
    if (j >= 32) {  // gapped events 2j, 2j+1 against 2j-64, 2j-63: s_{j-32}, e_{j-32}
      const uint64_t sq = (uint64_t)base + offs[j - 32];
      if (grp(s) == grp(sq) || grp(e) == grp(sq + lens[j - 32])) bad |= 2u;
    }
    if (j >= 64 && grp(e) == grp((uint64_t)base + offs[j - 64] + lens[j - 64])) bad |= 8u;  // e_j vs e_{j-64}
    if (j == 63 && grp(e) == grp(s0)) bad |= 8u;  // e_63 vs s_0 (event 0)
    if (none_left(bad)) {
      j += step;
      break;
    }
    const uint64_t us = (s - g.a0) >> kU, ue = (e - g.a0) >> kU;
    for (uint64_t u = ulo; u <= us; u++) first_ev[u] = (uint32_t)(2 * j);
    for (uint64_t u = us + 1; u <= ue; u++) first_ev[u] = (uint32_t)(2 * j + 1);
    if (j + 1 == n)
      for (uint64_t u = ue + 1; u <= g.units; u++) first_ev[u] = (uint32_t)(2 * n + 2);
  }
  for (; j < n; j += step) conf += grp_rec((uint64_t)base + offs[j], lens[j]);  // past an early stop
  __syncthreads();
  if (bad) atomicOr(&sh.bad, bad);
  if (gx) atomicAdd(&sh.gx, (unsigned long long)gx);
  if (conf) atomicAdd(&sh.conf, conf);
  __syncthreads();
  if (threadIdx.x == 0) {  // every slot written: no memset
    plan_bad[wg] = sh.bad;
    plan_gx[wg] = (long long)sh.gx;
    plan_conf[wg] = sh.conf;
  }
}

// sync (optional): the sort's barrier words (seg_sort), zeroed here for the
// k_seg_stream after this launch
template <uint32_t kU = kSegUnitLg>
__global__ __launch_bounds__(256) void k_seg_plan(const uint8_t *base, const uint64_t *__restrict__ offs,
                                                  const uint32_t *__restrict__ lens, uint64_t n, uint64_t max_units,
                                                  uint32_t *__restrict__ plan_bad, long long *__restrict__ plan_gx,
                                                  uint32_t *__restrict__ plan_conf, uint32_t *__restrict__ first_ev,
                                                  uint32_t *__restrict__ sync) {
  __shared__ SegPlanShared sh;
  if (sync && blockIdx.x == 0 && threadIdx.x < 3 + kSegSyncGroups) sync[threadIdx.x] = 0;
  seg_plan_body<kU>(base, offs, lens, n, max_units, blockIdx.x, gridDim.x, plan_bad, plan_gx, plan_conf, first_ev, sh);
}

// The stream over one event numbering (k_seg_plan): kGap, the 2n events of a
// sorted batch with gaps (each window lane loads off[] and len[] of its
// record: s_j = off, e_j = off + len); else the n + 1 events of a packed
// batch (off[] only, first_ev converted).  (Its timing-only builds -- rows
// XOR-folded, or no event work at all -- are in git history:
// tools/ab_hc_kernels.hip, up to commit 61a2e0e.)
template <uint32_t kMode, uint32_t kU, bool kView = false>
__device__ __forceinline__ void seg_stream_body(uint32_t *lds, uint32_t &s_next, const uint32_t (&col)[32],
                                                const uint8_t *base, const uint64_t *__restrict__ offs,
                                                const uint32_t *__restrict__ lens, uint64_t n, uint32_t lg_chunk,
                                                const uint32_t *__restrict__ first_ev, uint32_t *__restrict__ unit_raw,
                                                uint32_t *__restrict__ ev_h) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  constexpr bool kGap = kMode == kSegGapped;     // the 2n events s_j, e_j; gap bytes zeroed
  constexpr bool kEnds = kMode == kSegGapSmall;  // the n + 1 events s_0, e_0 .. e_{n-1}
  const uint32_t r4 = (lane & 31u) << 2;
  const uint32_t B0 = r4, B1 = r4 | 128u, B2 = 65536u | r4, B3 = 65536u | 128u | r4;
  const uint32_t S4base = kLdsMainBytes + ((lane & 3u) << 2);
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(c, B0, 0x0c020400u));
    const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(c, B1, 0x0c020500u));
    const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(c, B2, 0x0c020600u));
    const uint32_t t3 = lds_u32(lds, __builtin_amdgcn_perm(c, B3, 0x0c020700u));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, S4base + ((x & 255u) << 4));
    const uint32_t t1 = lds_u32(lds, S4base + 4096u + (((x >> 8) & 255u) << 4));
    const uint32_t t2 = lds_u32(lds, S4base + 8192u + (((x >> 16) & 255u) << 4));
    const uint32_t t3 = lds_u32(lds, S4base + 12288u + ((x >> 24) << 4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  // lane chunk (4 words) -> its raw CRC placed at the row end
  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    return matvec32(col, shift4(shift4(shift4(a, b_), c), d));
  };

  const uint32_t wave = uni(tid >> 6);
  const uint32_t slot = kFastLdsBytes / 4 + wave * 64;  // lds[slot + l]: event -> lane routing
  // (relaxed wavefront-scope atomics: ds_write/ds_read in program order, never
  // forwarded by the compiler across the other lanes' writes)
  auto slot_st = [&](uint32_t l, uint32_t v) {
    __hip_atomic_store(&lds[slot + l], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  };
  const SegGeo geo = seg_geo<kU>(base, offs, lens, n);
  const uint64_t M = geo.units;
  const uint64_t rhi = (geo.pend + 15) & ~15ull;  // loads past the span's last chunk return zeros
  const uint64_t G = gridDim.x;
  // chunks of 2^lg_chunk units, dealt to the workgroups round-robin (8 = 128
  // KiB: round 6's sweep on 2M records, 85.0 % against 83.2 % at round 2's 128
  // units -- the last round's 2 MiB chunks left a fifth of the workgroups
  // ~80 us behind the rest; 4 units 81.1 %, profiles/r6/r6q/), fewer
  // for short spans: every workgroup gets at least 4 chunks
  while (lg_chunk > 0 && (M >> lg_chunk) < G * 4) lg_chunk--;
  const uint32_t cmask = (1u << lg_chunk) - 1u;
  // each XCD's workgroups own neighbouring chunk slots (as k_crc_grp's kXcd)
  const uint64_t wgx = (G & 7u) == 0 ? (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  auto unit_of = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> lg_chunk) * G + wgx) << lg_chunk) | (k & cmask);
  };
  auto unit_rsrc = [&](uint64_t u) {
    const uint64_t U = geo.a0 + (u << kU);
    const uint64_t avail = u < M && rhi > U ? rhi - U : 0;
    return buf_range(reinterpret_cast<const void *>(U), (uint32_t)(avail < (1u << kU) ? avail : (1u << kU)));
  };
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  // the first event at or after unit u's start, in this body's numbering
  auto fev = [&](uint64_t u_) -> uint64_t {
    uint32_t f;  // (the plan's numbering is the 2n one)
    if constexpr (kView) {
      // the sorted view's first_ev, written earlier in this kernel (seg_sort):
      // hipcc makes a plain read of it a vector load whose vmcnt(0) drains the
      // row refills once a unit; a scalar load, waited for at once (lgkmcnt),
      // leaves them in flight (glc: past the scalar cache)
      const uint64_t pa = uni64(reinterpret_cast<uint64_t>(first_ev + u_));  // (SGPRs at every -O level)
      asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(f) : "s"(pa));
    } else {
      f = first_ev[u_];
    }
    if constexpr (kGap) return f;
    if constexpr (kEnds) return f ? (uint64_t)(f >> 1) + 1 : 0;
    return (uint64_t)((f + 1u) >> 1);
  };
  // window: the positions of events f .. f+63, one per lane (a group holds at most 64)
  struct Win {
    u32x2 o;
    uint32_t l;
  };
  auto win_issue = [&](uint64_t f) -> Win {
    Win w;
    if constexpr (kEnds) {  // event k >= 1 is e_{k-1} = off[k-1] + len[k-1]; event 0 is s_0
      const uint64_t r0 = f ? (f - 1 < n ? f - 1 : n) : 0;
      const uint64_t cnt = n - r0;
      const uint32_t rel = f ? lane : (lane ? lane - 1 : 0);
      const __amdgpu_buffer_rsrc_t ro = buf_range(offs + r0, (uint32_t)(cnt < 64 ? cnt * 8 : 512));
      const __amdgpu_buffer_rsrc_t rl = buf_range(lens + r0, (uint32_t)(cnt < 64 ? cnt * 4 : 256));
      w.o = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(ro, rel * 8u, 0, 0));
      w.l = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rl, rel * 4u, 0, 0);
      if (f == 0 && lane == 0) w.l = 0;
    } else if constexpr (!kGap) {
      const uint64_t fc = f < n ? f : n;
      const uint64_t cnt = n - fc;
      const __amdgpu_buffer_rsrc_t r = buf_range(offs + fc, (uint32_t)(cnt < 64 ? cnt * 8 : 512));
      w.o = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, lane * 8u, 0, 0));
      w.l = 0;
    } else {  // events f .. f+63 are s/e of at most 33 records from f >> 1
      const uint64_t r0 = (f >> 1) < n ? f >> 1 : n;
      const uint64_t cnt = n - r0;
      const uint32_t rel = (((uint32_t)f & 1u) + lane) >> 1;
      const __amdgpu_buffer_rsrc_t ro = buf_range(offs + r0, (uint32_t)(cnt < 33 ? cnt * 8 : 264));
      const __amdgpu_buffer_rsrc_t rl = buf_range(lens + r0, (uint32_t)(cnt < 33 ? cnt * 4 : 132));
      w.o = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(ro, rel * 8u, 0, 0));
      w.l = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rl, rel * 4u, 0, 0);
    }
    return w;
  };
  auto win_pos = [&](Win v, uint64_t f) -> uint64_t {
    const uint64_t j = f + lane;
    const uint64_t p = (uint64_t)base + (((uint64_t)v.o.y << 32) | v.o.x);
    if constexpr (kEnds) return j <= n ? p + v.l : ~0ull;
    if constexpr (!kGap) return j < n ? p : j == n ? geo.pend : ~0ull;
    return j < 2 * n ? p + ((j & 1u) ? v.l : 0u) : ~0ull;
  };

  uint64_t u = unit_of(wave);
  if (u >= M) return;
  uint64_t un = unit_of(kFastWaves + wave);
  uint32_t kv = 0;  // VGPR: the LDS hand-out result, read one unit later
  if (lane == 0) kv = atomicAdd(&s_next, 1u);
  uint64_t wfirst = fev(u);
  Win wraw = win_issue(wfirst);
  __amdgpu_buffer_rsrc_t rc = unit_rsrc(u);
  uint4 q0 = buf_load16(rc, lane * 16u), q1 = buf_load16(rc, 1024u + lane * 16u),
        q2 = buf_load16(rc, 2048u + lane * 16u), q3 = buf_load16(rc, 3072u + lane * 16u);
  // two empty stores, as the loop issues per group, so the loop's first waits
  // count the same VMEM ops as its later ones (hipcc takes the fewer)
  buf_store_u32(buf_range(ev_h, 0), 0u, lane * 4u);
  buf_store_u32(buf_range(unit_raw, 0), 0u, lane * 4u);
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, g = 0;
  uint32_t hv = 0;  // lane k: H of the group's event wfirst + k (stored once per group)
  uint32_t ur_pend = 0, ur_bytes = 0;  // the last unit's raw CRC, stored after the next group
  uint64_t u_pend = 0;
  // kGap: the stream hashes the span with every gap byte [e_{j-1}, s_j) zeroed.
  // Zeros do not change a raw CRC, so H(s_j) is H(e_{j-1}) shifted to s_j's row
  // (or 0 in a later unit) and the combine derives it: H is needed at the
  // record ends e_j (odd events) and at s_0 only -- one placement per record, as
  // a packed batch.  `ingap` (wave-uniform): the current row starts inside a
  // gap; at a unit's start, when its first event is a record start s_j (j > 0).
  auto gap_at = [&](uint64_t f) -> uint32_t { return kGap && f > 0 && f < 2 * n && !(f & 1u) ? 1u : 0u; };
  uint32_t ingap = gap_at(wfirst);

  // H at the events of the row starting at rs (uniform mask evm of window
  // lanes), from the streams c with the row already folded in: H(x) is the
  // finalize of the row folded with its bytes from x on zeroed, i.e. of
  // c ^ (w & ~m_x).  Rows with 1-2 events: one finalize per event.  More: the
  // lane-parallel form H = F(re) ^ R ^ X_L ^ Epre_L with E_l every lane chunk
  // placed at the row end, X its exclusive XOR scan, R = the row's raw CRC and
  // Epre_L the event lane's chunk cut at x, placed (one pass per event that
  // shares a lane chunk with an earlier one).
  auto keep = [](int q, int k) -> uint32_t {  // bytes of word k below byte q of the chunk
    const int nb = q - 4 * k;
    return nb >= 4 ? 0xFFFFFFFFu : nb <= 0 ? 0u : (1u << (8 * nb)) - 1u;
  };
  auto events = [&](const uint4 w, uint64_t rs, uint64_t wpos, uint64_t evm) {
    if (__popcll(evm) <= 2) {
      for (uint64_t m = evm; m; m &= m - 1) {
        const uint32_t k = (uint32_t)__builtin_ctzll(m);
        const uint32_t rel = uni((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(wpos - rs), k));
        const int L = (int)(rel >> 4), q = lane == (uint32_t)L ? (int)(rel & 15u) : lane < (uint32_t)L ? 16 : 0;
        const uint32_t h = wave_xor(place(c0 ^ (w.x & ~keep(q, 0)), c1 ^ (w.y & ~keep(q, 1)),
                                          c2 ^ (w.z & ~keep(q, 2)), c3 ^ (w.w & ~keep(q, 3))));
        hv = lane == k ? h : hv;
      }
      return;
    }
    const uint32_t fre = wave_xor(place(c0, c1, c2, c3));  // raw(unit .. re)
    const uint32_t e = place(w.x, w.y, w.z, w.w);
    uint32_t x = e;  // inclusive XOR scan over the lanes
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(x, d);
      if (lane >= d) x ^= t;
    }
    const uint32_t base_h = fre ^ uni((uint32_t)__builtin_amdgcn_readlane((int)x, 63));  // F(re) ^ R
    x ^= e;                                                                              // exclusive
    const uint32_t rel = (uint32_t)(wpos - rs);  // event lanes: < 1024
    const uint32_t L = rel >> 4;
    const uint32_t Lp = __shfl_up(L, 1);
    const uint64_t same = __ballot(lane > 0 && Lp == L) & evm & (evm << 1);
    uint64_t rem = evm;
    while (rem) {  // one pass per event sharing a lane chunk with an earlier one
      const uint64_t sel = rem & ~((rem << 1) & same);
      slot_st(lane, 0xFFFFFFFFu);
      if ((sel >> lane) & 1u) slot_st(L, lane | ((rel & 15u) << 8));
      const uint32_t sv = __hip_atomic_load(&lds[slot + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      const bool has = sv != 0xFFFFFFFFu;
      const int q = has ? (int)(sv >> 8) : 0;
      const uint32_t ep = place(w.x & keep(q, 0), w.y & keep(q, 1), w.z & keep(q, 2), w.w & keep(q, 3));
      const uint32_t hl = __shfl(base_h ^ x ^ ep, (int)L);  // event lane k <- its chunk's lane L
      hv = (sel >> lane) & 1u ? hl : hv;
      rem &= ~sel;
    }
  };
  // a row: fold it, its events, then its register's refill.  (Round 3 issued
  // the refill before the events, from a copy of the row, to keep 4 loads in
  // flight through the event work; the copy's 4 v_mov a row cost more than
  // the wait under sustained launches, where the clock is what the work
  // leaves: +0.55 points, profiles/r4/r4m/.)  The row as one 128-bit asm
  // operand where it is folded keeps the loop-carried row in its load's
  // register tuple: without it small changes elsewhere made hipcc copy the
  // rows at the loop latch, which waits for the refills.
  auto row = [&](uint4 &q, uint64_t rs, uint64_t wpos, __amdgpu_buffer_rsrc_t rn, uint32_t no) {
    typedef unsigned int r32x4 __attribute__((ext_vector_type(4)));
    r32x4 qq = __builtin_bit_cast(r32x4, q);
    asm volatile("" : "+v"(qq));
    uint4 w = __builtin_bit_cast(uint4, qq);
    const uint64_t evm = __ballot(wpos >= rs && wpos < rs + 1024u);
    uint64_t evh = evm;  // the events that need H
    if constexpr (kGap) {
      // window lanes k with wfirst + k odd: record ends (they open a gap; the
      // even ones, record starts, close it)
      const uint64_t ends = (wfirst & 1u) ? 0x5555555555555555ull : 0xAAAAAAAAAAAAAAAAull;
      evh = evm & (ends | (wfirst == 0 ? 1ull : 0ull));
      if (ingap || evm) {
        uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0, lo = 0;
        uint32_t open = ingap;
        auto zero = [&](uint32_t a, uint32_t b) {  // row bytes [a, b)
          const int qa = min(max((int)a - (int)(16u * lane), 0), 16), qb = min(max((int)b - (int)(16u * lane), 0), 16);
          g0 |= keep(qb, 0) & ~keep(qa, 0);
          g1 |= keep(qb, 1) & ~keep(qa, 1);
          g2 |= keep(qb, 2) & ~keep(qa, 2);
          g3 |= keep(qb, 3) & ~keep(qa, 3);
        };
        for (uint64_t m = evm; m; m &= m - 1) {
          const uint32_t k = (uint32_t)__builtin_ctzll(m);
          const uint32_t rel = uni((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(wpos - rs), k));
          if ((ends >> k) & 1u) {
            lo = rel;
            open = 1;
          } else if (open) {
            zero(lo, rel);
            open = 0;
          }
        }
        if (open) zero(lo, 1024u);
        ingap = open;
        w.x &= ~g0;
        w.y &= ~g1;
        w.z &= ~g2;
        w.w &= ~g3;
      }
    }
    c0 = row_step(c0, w.x);
    c1 = row_step(c1, w.y);
    c2 = row_step(c2, w.z);
    c3 = row_step(c3, w.w);
    asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
    if (evh) events(w, rs, wpos, evh);
    __builtin_amdgcn_sched_barrier(0);
    q = buf_load16(rn, no);
    __builtin_amdgcn_sched_barrier(0);
  };

  for (;;) {
    const uint64_t gs = geo.a0 + (u << kU) + ((uint64_t)g << 12);
    const uint64_t wpos = win_pos(wraw, wfirst);
    const bool lastg = g == (1u << (kU - 12)) - 1u;  // the unit's last 4 KiB group
    // the next group: this unit's, or unit un's first; its events' window
    const uint32_t gcnt = (uint32_t)__popcll(__ballot(wpos < gs + 4096u));  // the group's events
    const uint64_t nf = lastg ? fev(un < M ? un : M) : wfirst + gcnt;
    const __amdgpu_buffer_rsrc_t rn = lastg ? unit_rsrc(un) : rc;
    const uint32_t no = lastg ? lane * 16u : ((g + 1) << 12) + lane * 16u;
    // each refill pinned right after its row's fold and events (sched
    // barriers, as k_crc_grp's kPin): hipcc otherwise hoists it into a fresh
    // register and copies that at the loop latch, which waits for the load
    wraw = win_issue(nf);
    row(q0, gs, wpos, rn, no);
    row(q1, gs + 1024u, wpos, rn, no + 1024u);
    row(q2, gs + 2048u, wpos, rn, no + 2048u);
    row(q3, gs + 3072u, wpos, rn, no + 3072u);
    // the group's event words and the previous unit's raw CRC (if one is
    // pending): two buffer stores every group, straight-line code (a store
    // behind a branch makes hipcc's vmcnt waits count the path without it)
    buf_store_u32(buf_range(ev_h + wfirst, gcnt * 4u), hv, lane * 4u);
    buf_store_u32(buf_range(unit_raw + u_pend, ur_bytes), ur_pend, lane * 4u);
    ur_bytes = 0;
    wfirst = nf;
    if (lastg) {
      ur_pend = wave_xor(place(c0, c1, c2, c3));
      u_pend = u;
      ur_bytes = 4;
      if (un >= M) {
        buf_store_u32(buf_range(unit_raw + u_pend, 4u), ur_pend, lane * 4u);
        return;
      }
      u = un;
      rc = rn;
      g = 0;
      c0 = c1 = c2 = c3 = 0;
      ingap = gap_at(nf);
      un = unit_of(uni(kv));
      if (lane == 0) kv = atomicAdd(&s_next, 1u);
    } else {
      g++;
    }
  }
}

// ---------------------------------------------------------------------------
// The sorted view of an unsorted batch (round 6; DESIGN.md
// 4.2b).  Records listed out of order (config 5's records in a permuted order:
// 66 % of 8 TB/s on k_crc_any's work, against 83 % for the same records in
// order on the stream) are sorted by start offset inside k_seg_stream, whose
// persistent grid (one workgroup per CU) meets at grid barriers between the
// phases; the plan of the sorted view is made there too, and the stream then
// runs over it.  k_seg_combine reads the sorted arrays and writes each word
// through the permutation.  The sort is a bucket sort by 16 KiB unit (the
// stream's own unit): count per unit (atomics), scan, scatter by arrival,
// then each record's rank among its unit's records (a unit holds at most 256
// records of >= 64 B; more than kSegSortMaxBucket in one unit: no sort).
// Phases, over the workspace arrays of SegSort (its own first_ev: the batch's
// stays unwritten in this kernel, so the unsorted stream keeps reading it with
// scalar loads) and the stream's unit_raw (unit starts; the stream rewrites it).
struct SegSort {
  uint4 *reca, *recb;       // n each: (key = start - A0, batch index, length) by coarse bucket, then by unit
  uint64_t *off;            // n: the sorted view's offsets
  uint32_t *arr;            // n: each record's arrival rank in its unit (recA order)
  uint32_t *len;            // n: the sorted view's lengths
  uint32_t *perm;           // n: sorted position -> batch index
  uint32_t *hc;             // kSegSortNbcMax x kSegSortMaxWgs: tile counts per coarse bucket, then offsets
  uint32_t *tc, *tb;        // kSegSortNbcMax each: coarse bucket totals and bases
  unsigned long long *wlo, *whi;  // kSegSortMaxWgs: per-workgroup lowest start / highest end
  uint32_t *sync;           // 18 words (zeroed by k_seg_plan): the first barrier, the others' root and 16 group counters
  uint32_t *fev;            // max_units + 1: the sorted view's first_ev
  uint32_t spins;           // the first barrier's bound (kSegSyncSpins; HC_SEG_SYNC_SPINS, a test hook)
  uint32_t ucmax;           // units per coarse bucket at most (kSegSortUcMax; HC_SEG_SORT_UC, a test hook)
};
constexpr uint32_t kSegSortedBit = 8;        // the mode word of a sorted view: its mode | 8
// Phase clock of the last sort (hc_debug_seg_prof): workgroup 0's s_memrealtime
// (100 MHz): [0] the stream's start, [1] its prologue, [2] the key range and
// the residency check, [3..7] the sort's barriers (A1, A2, A3, B, P5), [10] P6,
// [14] / [15] the sorted body's start / end; inside B, workgroup 0's own bucket:
// [8] counted, [9] scanned, [11] scattered, [12] ranked.  One store each by one thread.
__device__ unsigned long long g_seg_prof[16];
__device__ __forceinline__ void seg_prof(uint32_t k) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && k < 16) g_seg_prof[k] = __builtin_amdgcn_s_memrealtime();
}
constexpr uint32_t kSegSortMaxBucket = 1024; // most records one 16 KiB unit may start (zero-length ones)
constexpr uint32_t kSegSortMaxWgs = 1024;    // the stream's largest grid with a sort
constexpr uint32_t kSegSortUcMax = 32768;    // units per coarse bucket: the LDS counters of phase B (128 KiB)
constexpr uint32_t kSegSortNbcMax = 4096;    // coarse buckets (2 LDS words each in phase A)
constexpr uint32_t kSegSyncAbort = 1u << 31;
constexpr uint64_t kSegSortLdsWords = kFastLdsBytes / 4 + kFastWaves * 64;  // the stream's LDS, the sort's scratch
static_assert(kSegSortUcMax + 1 <= kSegSortLdsWords, "phase B's unit counters fit the sort's LDS");

// workspace (u32 words): the mode flag (64 words: word 0 the mode, words 1-18
// the sort's barrier words), plan_bad[kSegPlanMaxWgs], plan_gx[kSegPlanMaxWgs]
// (int64), plan_conf[kSegPlanMaxWgs], first_ev[max_units + 1],
// unit_raw[max_units], ev_h[2n + 1] (the gapped numbering's 2n events; a
// packed batch uses n + 1); with a sort, SegSort's arrays after it.
struct SegWs {
  uint32_t *flag, *plan_bad, *plan_conf, *first_ev, *unit_raw, *ev_h;
  long long *plan_gx;
  SegSort ss;
  uint64_t bytes;
};
__host__ __device__ __forceinline__ SegWs seg_ws_layout(uint32_t *ws, uint64_t n, uint64_t max_units, bool sort) {
  SegWs w{};
  uint64_t o = 0;  // bytes
  auto take = [&](uint64_t bytes, uint64_t align) {
    o = (o + align - 1) & ~(align - 1);
    uint8_t *p = ws ? reinterpret_cast<uint8_t *>(ws) + o : nullptr;
    o += bytes;
    return p;
  };
  w.flag = reinterpret_cast<uint32_t *>(take(4 * 64, 4));
  w.plan_bad = reinterpret_cast<uint32_t *>(take(4ull * kSegPlanMaxWgs, 4));
  w.plan_gx = reinterpret_cast<long long *>(take(8ull * kSegPlanMaxWgs, 8));
  w.plan_conf = reinterpret_cast<uint32_t *>(take(4ull * kSegPlanMaxWgs, 4));
  w.first_ev = reinterpret_cast<uint32_t *>(take(4 * (max_units + 1), 4));
  w.unit_raw = reinterpret_cast<uint32_t *>(take(4 * max_units, 4));
  w.ev_h = reinterpret_cast<uint32_t *>(take(4 * (2 * n + 1), 4));
  if (sort) {
    w.ss.reca = reinterpret_cast<uint4 *>(take(16 * n, 16));
    w.ss.recb = reinterpret_cast<uint4 *>(take(16 * n, 16));
    w.ss.off = reinterpret_cast<uint64_t *>(take(8 * n, 8));
    w.ss.arr = reinterpret_cast<uint32_t *>(take(4 * n, 4));
    w.ss.len = reinterpret_cast<uint32_t *>(take(4 * n, 4));
    w.ss.perm = reinterpret_cast<uint32_t *>(take(4 * n, 4));
    w.ss.hc = reinterpret_cast<uint32_t *>(take(4ull * kSegSortNbcMax * kSegSortMaxWgs, 4));
    w.ss.tc = reinterpret_cast<uint32_t *>(take(4ull * kSegSortNbcMax, 4));
    w.ss.tb = reinterpret_cast<uint32_t *>(take(4ull * kSegSortNbcMax, 4));
    w.ss.wlo = reinterpret_cast<unsigned long long *>(take(8ull * kSegSortMaxWgs, 8));
    w.ss.whi = reinterpret_cast<unsigned long long *>(take(8ull * kSegSortMaxWgs, 8));
    w.ss.fev = reinterpret_cast<uint32_t *>(take(4 * (max_units + 1), 4));
    w.ss.sync = w.flag + 1;
    w.ss.spins = 0;
    w.ss.ucmax = 0;
  }
  w.bytes = (o + 7) & ~7ull;
  return w;
}

// The first grid barrier, also the check that the whole grid is resident (a
// grid barrier needs every workgroup on a CU at once: k_seg_stream takes one CU
// each).  A workgroup that waits `limit` polls (kSegSyncSpinsDefault: s_sleep + an L2
// round trip each, ~0.1-0.3 s) sets the abort bit by a
// CAS on the counter word, which fails if the last workgroup arrived meanwhile;
// so either every workgroup passes or every one sees the abort, and none waits
// on a later barrier for a workgroup that left.  The later barriers need no
// bound: every workgroup that passed the first is resident until it exits.
// Fences: the workgroup barrier leaves every wave's stores acknowledged by the
// XCD's L2; ONE agent-scope release (thread 0) then writes that L2 back, and
// one acquire invalidates the CU's L1 and the L2 before the second barrier
// releases the waves.  (The first build fenced in every thread: 16 L2
// writebacks per workgroup per barrier.)
__device__ __forceinline__ bool seg_sync_first(uint32_t *w, uint32_t G, uint32_t limit, uint32_t &s_ok) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    uint32_t v = __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    uint32_t spins = 0;
    bool ok;
    for (;;) {
      if (v & kSegSyncAbort) {
        ok = false;
        break;
      }
      if (v >= G) {
        ok = true;
        break;
      }
      if (++spins > limit) {
        uint32_t expect = v;
        if (__hip_atomic_compare_exchange_strong(w, &expect, v | kSegSyncAbort, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          ok = false;
          break;
        }
        v = expect;  // the word moved: an arrival or another workgroup's abort
        continue;
      }
      __builtin_amdgcn_s_sleep(2);
      v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_ok = ok ? 1u : 0u;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  return s_ok != 0;
}
// The later barriers, k = 1, 2, ...: a two-level counter tree.  Workgroup w
// arrives on sub[w % 16]; the last arrival of a group raises root; everyone
// polls root.  (One counter for all 256 workgroups serialised 256 device-scope
// atomics on one address per barrier, ~15-20 us each.)  Counters only grow: a
// group of g workgroups has seen k g arrivals after barrier k.
__device__ __forceinline__ void seg_sync(uint32_t *root, uint32_t *sub, uint32_t k) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t G = gridDim.x, ng = G < kSegSyncGroups ? G : kSegSyncGroups, grp = blockIdx.x % ng;
    const uint32_t gsize = (G - grp + ng - 1) / ng;
    const uint32_t v = __hip_atomic_fetch_add(sub + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (v == k * gsize) __hip_atomic_fetch_add(root, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k * ng) __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// Workgroup reductions / scan over blockDim.x threads (<= 1024), through 16 +
// 16 shared words; each call ends with a barrier, so calls can follow each other.
struct SegRed {
  uint32_t w[kFastWaves], w2[kFastWaves];
  unsigned long long q[kFastWaves];
};
__device__ __forceinline__ uint32_t block_max_u32(uint32_t v, SegRed &r) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
  if ((threadIdx.x & 63u) == 0) r.w[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) t = max(t, r.w[k]);
  __syncthreads();
  return t;
}
__device__ __forceinline__ uint32_t block_or_u32(uint32_t v, SegRed &r) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d);
  if ((threadIdx.x & 63u) == 0) r.w[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) t |= r.w[k];
  __syncthreads();
  return t;
}
__device__ __forceinline__ long long block_sum_i64(long long v, SegRed &r) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  if ((threadIdx.x & 63u) == 0) r.q[threadIdx.x >> 6] = (unsigned long long)v;
  __syncthreads();
  long long t = 0;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) t += (long long)r.q[k];
  __syncthreads();
  return t;
}
__device__ __forceinline__ unsigned long long block_min_u64(unsigned long long v, SegRed &r) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(v, d);
    v = o < v ? o : v;
  }
  if ((threadIdx.x & 63u) == 0) r.q[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long t = ~0ull;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) t = r.q[k] < t ? r.q[k] : t;
  __syncthreads();
  return t;
}
__device__ __forceinline__ unsigned long long block_max_u64(unsigned long long v, SegRed &r) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(v, d);
    v = o > v ? o : v;
  }
  if ((threadIdx.x & 63u) == 0) r.q[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long t = 0;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) t = r.q[k] > t ? r.q[k] : t;
  __syncthreads();
  return t;
}
// exclusive prefix of v over the threads in order; *total = the sum
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, SegRed &r, uint32_t &total) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(x, d);
    if (lane >= d) x += t;
  }
  if (lane == 63) r.w[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) {
    if (k < (threadIdx.x >> 6)) before += r.w[k];
    tot += r.w[k];
  }
  __syncthreads();
  total = tot;
  return before + x - v;
}

// OR of bad, sums of gx and conf over the workgroup, in one exchange (the
// stream's prologue: round 6's first build took 10 us there with one
// reduction per value)
__device__ __forceinline__ void seg_block_reduce3(uint32_t &bad, long long &gx, uint32_t &conf, SegRed &r) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    bad |= __shfl_xor(bad, d);
    gx += __shfl_xor(gx, d);
    conf += __shfl_xor(conf, d);
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 0) {
    r.w[w] = bad;
    r.q[w] = (unsigned long long)gx;
    r.w2[w] = conf;
  }
  __syncthreads();
  bad = 0;
  gx = 0;
  conf = 0;
  for (uint32_t k = 0; k < (blockDim.x >> 6); k++) {
    bad |= r.w[k];
    gx += (long long)r.q[k];
    conf += r.w2[k];
  }
  __syncthreads();
}

// The sort and the plan of the sorted view (every workgroup of the grid; the
// caller checked that the key range fits max_units units).  Returns the sorted
// view's stream mode, or kSegFallback (the grid was not resident, a unit held
// too many records, or the sorted records overlap / are refused by the plan):
// uniform over the grid.
template <uint32_t kU>
__device__ uint32_t seg_sort(const uint8_t *base, const uint64_t *__restrict__ offs,
                             const uint32_t *__restrict__ lens, uint64_t n, uint64_t max_units, const SegSort &ss,
                             uint32_t *scratch, uint32_t *__restrict__ plan_bad,
                             long long *__restrict__ plan_gx, uint32_t *__restrict__ plan_conf, SegPlanShared &psh,
                             SegRed &red, uint32_t &s_ok) {
  const uint32_t G = gridDim.x, wg = blockIdx.x, T = blockDim.x, tid = threadIdx.x;
  const uint64_t gstep = (uint64_t)G * T, g0 = (uint64_t)wg * T + tid;
  // P-1: the key range (lowest start, highest end), per workgroup, then over the grid
  uint64_t lo = ~0ull, hi = 0;
  for (uint64_t j = g0; j < n; j += gstep) {
    const uint64_t s = (uint64_t)base + offs[j], e = s + lens[j];
    lo = s < lo ? s : lo;
    hi = e > hi ? e : hi;
  }
  lo = block_min_u64(lo, red);
  hi = block_max_u64(hi, red);
  if (tid == 0) {
    ss.wlo[wg] = lo;
    ss.whi[wg] = hi;
  }
  if (!seg_sync_first(ss.sync, G, ss.spins, s_ok)) return kSegFallback;
  uint32_t phase = 0;
  auto sync = [&]() {
    seg_sync(ss.sync + 1, ss.sync + 2, ++phase);
    seg_prof(2 + phase);  // 3: A1 done, 4: A2, 5: A3, 6: B, 7: P5
  };
  seg_prof(2);  // the key range + the residency check
  lo = ~0ull;
  hi = 0;
  for (uint32_t k = tid; k < G; k += T) {
    lo = ss.wlo[k] < lo ? ss.wlo[k] : lo;
    hi = ss.whi[k] > hi ? ss.whi[k] : hi;
  }
  const uint64_t smin = uni64(block_min_u64(lo, red)), emax = uni64(block_max_u64(hi, red));
  const uint64_t A0 = smin & ~1023ull;
  // (uniform over the grid: every workgroup read the same slots)
  if (smin > emax || ((emax - A0) >> kU) + 1 > max_units) return kSegFallback;
  const uint64_t NB = ((emax - A0) >> kU) + 1;
  // nbc coarse buckets of UC units each, one owner workgroup a bucket (d % G)
  const uint64_t ucmax = ss.ucmax ? (ss.ucmax < kSegSortUcMax ? ss.ucmax : kSegSortUcMax) : kSegSortUcMax;
  const uint64_t m = (NB + (uint64_t)G * ucmax - 1) / ((uint64_t)G * ucmax);
  if (m * G > kSegSortNbcMax) return kSegFallback;  // (a span of more than 2^40 bytes)
  const uint32_t nbc = (uint32_t)m * G;
  const uint64_t UC = (NB + nbc - 1) / nbc;
  const uint64_t off0 = A0 - (uint64_t)base;
  // a record's coarse bucket: its unit / UC in 32 bits (units < 2^32; a 64-bit
  // division by a run-time value is a long call per record)
  const uint32_t uc32 = (uint32_t)UC;
  auto bucket_of = [&](uint64_t key) -> uint32_t { return (uint32_t)(key >> kU) / uc32; };
  // A: the workgroup's tile of the batch (contiguous: coalesced reads)
  const uint64_t tile = (n + G - 1) / G;
  const uint64_t j_lo = (uint64_t)wg * tile < n ? (uint64_t)wg * tile : n, j_hi = j_lo + tile < n ? j_lo + tile : n;
  uint32_t *hist = scratch, *lbase = scratch + kSegSortNbcMax;  // LDS
  // A1: histogram of the tile over the coarse buckets (LDS atomics)
  for (uint32_t d = tid; d < nbc; d += T) hist[d] = 0;
  __syncthreads();
  for (uint64_t j = j_lo + tid; j < j_hi; j += T)
    atomicAdd(&hist[bucket_of((uint64_t)base + offs[j] - A0)], 1u);
  __syncthreads();
  for (uint32_t d = tid; d < nbc; d += T) ss.hc[(uint64_t)d * G + wg] = hist[d];
  sync();  // 3
  // A2: bucket d's offsets of the workgroups' tiles (exclusive, in place) and its total
  for (uint32_t d = wg; d < nbc; d += G) {
    const uint32_t v = tid < G ? ss.hc[(uint64_t)d * G + tid] : 0u;
    uint32_t tot = 0;
    const uint32_t ex = block_excl_scan_u32(v, red, tot);
    if (tid < G) ss.hc[(uint64_t)d * G + tid] = ex;
    if (tid == 0) ss.tc[d] = tot;
  }
  sync();  // 4
  // A3: the buckets' bases (every workgroup: a scan of the nbc totals), then the
  // tile's records to recA, each at its bucket's base + the tile's offset + its
  // arrival rank in the tile (LDS atomics)
  {
    const uint32_t per = (nbc + T - 1) / T, d0 = tid * per, d1 = d0 + per < nbc ? d0 + per : nbc;
    uint32_t sum = 0;
    for (uint32_t d = d0; d < d1; d++) sum += ss.tc[d];
    uint32_t tot = 0;
    uint32_t run = block_excl_scan_u32(sum, red, tot);
    for (uint32_t d = d0; d < d1; d++) {
      if (wg == 0) ss.tb[d] = run;  // (phase B reads the bases there: its counters reuse this LDS)
      lbase[d] = run + ss.hc[(uint64_t)d * G + wg];
      hist[d] = 0;
      run += ss.tc[d];
    }
  }
  __syncthreads();
  for (uint64_t j = j_lo + tid; j < j_hi; j += T) {
    const uint64_t key = (uint64_t)base + offs[j] - A0;
    const uint32_t d = bucket_of(key);
    const uint32_t pos = lbase[d] + atomicAdd(&hist[d], 1u);
    ss.reca[pos] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), (uint32_t)j, lens[j]);
  }
  sync();  // 5
  // B: each owned bucket by unit, in LDS counters: count (arrival ranks), scan,
  // scatter to recb inside the bucket's range, then each record's rank among its
  // unit's records (start, then batch index: zero-length records may share a
  // start) -> the sorted arrays.  Every access stays in the bucket's range.
  uint32_t *ucnt = scratch;  // UC + 1 words (the A arrays are no longer needed)
  uint32_t too_many = 0;
  for (uint32_t d = wg; d < nbc; d += G) {
    const uint64_t p0 = ss.tb[d], pc = ss.tc[d];
    const uint64_t u0 = (uint64_t)d * UC, nu = u0 < NB ? (NB - u0 < UC ? NB - u0 : UC) : 0;
    __syncthreads();  // (the previous bucket's readers of ucnt are done)
    for (uint64_t u = tid; u <= nu; u += T) ucnt[u] = 0;
    __syncthreads();
    for (uint64_t p = p0 + tid; p < p0 + pc; p += T) {
      const uint4 r = ss.reca[p];
      const uint64_t key = ((uint64_t)r.y << 32) | r.x;
      ss.arr[p] = atomicAdd(&ucnt[(key >> kU) - u0], 1u);
    }
    __syncthreads();
    seg_prof(8);
    {  // exclusive scan of ucnt[0 .. nu) in place; ucnt[nu] = the total
      const uint32_t per = (uint32_t)((nu + T - 1) / T);
      const uint64_t a0 = (uint64_t)tid * per, a1 = a0 + per < nu ? a0 + per : nu;
      uint32_t sum = 0, mx = 0;
      for (uint64_t u = a0; u < a1; u++) {
        sum += ucnt[u];
        mx = ucnt[u] > mx ? ucnt[u] : mx;
      }
      uint32_t tot = 0;
      uint32_t run = block_excl_scan_u32(sum, red, tot);
      too_many |= block_max_u32(mx, red) > kSegSortMaxBucket ? 1u : 0u;
      for (uint64_t u = a0; u < a1; u++) {
        const uint32_t c = ucnt[u];
        ucnt[u] = run;
        run += c;
      }
      if (tid == 0) ucnt[nu] = tot;
    }
    __syncthreads();
    seg_prof(9);
    if (too_many) continue;  // (workgroup-uniform; the grid learns it below)
    for (uint64_t p = p0 + tid; p < p0 + pc; p += T) {
      const uint4 r = ss.reca[p];
      const uint64_t key = ((uint64_t)r.y << 32) | r.x;
      ss.recb[p0 + ucnt[(key >> kU) - u0] + ss.arr[p]] = r;
    }
    __syncthreads();
    seg_prof(11);
    // ranks: against LDS copies of the bucket's keys (from the bucket's first
    // unit, 32 bits) and batch indices when they fit beside the unit counts,
    // else against recb itself (one L2 round trip per record of the unit)
    const uint64_t ub = u0 << kU;
    uint32_t *kk = ucnt + nu + 1, *ii = kk + pc;
    const bool in_lds = nu + 1 + 2 * pc <= kSegSortLdsWords;
    if (in_lds) {
      for (uint64_t p = tid; p < pc; p += T) {
        const uint4 r = ss.recb[p0 + p];
        kk[p] = (uint32_t)((((uint64_t)r.y << 32) | r.x) - ub);
        ii[p] = r.z;
      }
      __syncthreads();
    }
    for (uint64_t p = p0 + tid; p < p0 + pc; p += T) {
      const uint4 me = ss.recb[p];
      const uint64_t key = ((uint64_t)me.y << 32) | me.x;
      const uint64_t u = (key >> kU) - u0;
      const uint32_t s0 = ucnt[u], c = ucnt[u + 1] - s0;
      uint32_t rank = 0;
      if (in_lds) {
        const uint32_t mk = (uint32_t)(key - ub);
        for (uint32_t q = 0; q < c; q++) {
          const uint32_t kq = kk[s0 + q];
          rank += (kq < mk || (kq == mk && ii[s0 + q] < me.z)) ? 1u : 0u;
        }
      } else {
        for (uint32_t q = 0; q < c; q++) {
          const uint4 o = ss.recb[p0 + s0 + q];
          const uint64_t kq = ((uint64_t)o.y << 32) | o.x;
          rank += (kq < key || (kq == key && o.z < me.z)) ? 1u : 0u;
        }
      }
      const uint64_t pos = p0 + s0 + rank;
      ss.off[pos] = key + off0;
      ss.len[pos] = me.w;
      ss.perm[pos] = me.z;
    }
    __syncthreads();
    seg_prof(12);
  }
  if (too_many && tid == 0) __hip_atomic_fetch_or(ss.sync + 2 + kSegSyncGroups, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
  sync();  // 6
  if (__hip_atomic_load(ss.sync + 2 + kSegSyncGroups, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return kSegFallback;  // a unit starting more than kSegSortMaxBucket records (every workgroup reads the flag)
  // P5: the plan of the sorted view (first_ev, the slots 0 .. G-1)
  seg_plan_body<kU>(base, ss.off, ss.len, n, max_units, wg, G, plan_bad, plan_gx, plan_conf, ss.fev, psh);
  sync();
  // P6: its mode, as the prologue chooses one (no k_crc_grp: this batch is not all its blocks)
  uint32_t bad = 0;
  long long gx = 0;
  for (uint32_t k = tid; k < G; k += T) {
    bad |= plan_bad[k];
    gx += plan_gx[k];
  }
  bad = block_or_u32(bad, red);
  gx = block_sum_i64(gx, red);
  seg_prof(10);
  return !(bad & 1u)                ? kSegPacked
         : !(bad & 12u) && gx <= 0  ? kSegGapSmall
         : !(bad & 2u) && gx <= 0   ? kSegGapped
                                    : kSegFallback;
}

// The prologue reduces the plan's slots beside the table fill: packed when no
// workgroup found the batch unpacked, else gapped when none found it out of
// order and the gap bytes are at most a quarter of the payload, else the
// fallback (all exit; k_seg_combine runs k_crc_any's work).  Workgroup 0 stores
// the mode for the combine.
template <uint32_t kU = kSegUnitLg>
__global__ __launch_bounds__(kFastThreads) void k_seg_stream(const uint8_t *base, const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint32_t lg_chunk, uint32_t *__restrict__ plan_bad,
                                                            long long *__restrict__ plan_gx,
                                                            uint32_t *__restrict__ plan_conf, uint32_t plan_wgs,
                                                            uint32_t allow_grp,
                                                            uint32_t *__restrict__ flag,
                                                            const uint32_t *__restrict__ first_ev,
                                                            uint32_t *__restrict__ unit_raw, uint32_t *__restrict__ ev_h,
                                                            const DeviceTables *__restrict__ tables,
                                                            uint64_t max_units, uint32_t *__restrict__ ws,
                                                            uint32_t sort_on, uint32_t sync_spins, uint32_t sort_uc) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kSegSortLdsWords];  // (the tables + the event slots)
  __shared__ uint32_t s_next, s_ok;
  __shared__ SegRed red;
  __shared__ SegPlanShared psh;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  if (tid == 0) s_next = 2 * kFastWaves;  // indices 0 .. 2W-1 are dealt statically below
  seg_prof(0);
  uint32_t bad = 0, conf = 0;
  long long gx = 0;
  for (uint32_t i = tid; i < plan_wgs; i += kFastThreads) {
    bad |= plan_bad[i];
    gx += plan_gx[i];
    conf += plan_conf[i];
  }
  // one exchange for the three (readfirstlane: hipcc then knows the results are
  // uniform; else every address the stream body forms from them is a VGPR)
  seg_block_reduce3(bad, gx, conf, red);
  const uint32_t unpacked = uni(bad & 1u), unsorted = uni(bad & 2u), not_small = uni(bad & 12u);
  const long long gsum = (long long)uni64((uint64_t)gx);
  const uint64_t csum = uni(conf);
  // k_crc_grp when every record is one of its blocks (16-B aligned 4 KiB
  // multiples) in a large batch, whatever their order: ahead of the stream's
  // own modes, whose event work at 4 KiB records costs more than the hand-out
  // (1M x 4 KiB, TB/s: packed 4.65 vs 5.73, 16-B gaps 4.37 vs 5.51, 1 KiB gaps
  // 3.75 vs 6.31, tools/seg_aligned_probe.py, profiles/r5/r5s/; ADVICE r4: the
  // per-record body ran 57-62 % on them).  Else the stream; else k_crc_any's
  // work in the combine.
  uint32_t mode = allow_grp && csum == n      ? kSegFallbackGrp
                  : !unpacked                 ? kSegPacked
                  : !not_small && gsum <= 0   ? kSegGapSmall
                  : !unsorted && gsum <= 0    ? kSegGapped
                                              : kSegFallback;
  if (blockIdx.x == 0 && tid == 0) *flag = mode;  // read by k_seg_combine
  // a batch the stream refuses, given a sort workspace (launch_seg: from
  // sort_min records) whose key range fits the unit arrays: its sorted view
  bool sorted = false;
  seg_prof(1);  // the prologue's reductions done
  // (the sort's pointers come from the workspace base here, not as kernel
  // arguments: live across the kernel, they pushed the unsorted small-gap
  // loop's SGPRs into spills -- 16 more reloads a group, -0.75 points)
  SegSort ss{};
  if (mode == kSegFallback && sort_on && gridDim.x <= kSegSortMaxWgs) {
    ss = seg_ws_layout(ws, n, max_units, true).ss;
    ss.spins = sync_spins;
    ss.ucmax = sort_uc;
    mode = uni(seg_sort<kU>(base, offs, lens, n, max_units, ss, lds, plan_bad, plan_gx, plan_conf, psh, red, s_ok));
    sorted = mode != kSegFallback;
    if (sorted && blockIdx.x == 0 && tid == 0) *flag = mode | kSegSortedBit;
  }
  // a fallback has no stream work: no table fill (r5: the fill was 8 of the
  // 9 us this kernel took when k_crc_grp took the batch)
  if (mode == kSegFallback || mode == kSegFallbackGrp) return;
  fill_crc_tables(lds, tables, tid, kFastThreads);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  __syncthreads();
  // (two call sites, not one over a pointer chosen at run time: through the
  // chosen pointer hipcc spilled 64 VGPRs of the stream loops)
  auto run = [&](auto view, const uint64_t *__restrict__ o, const uint32_t *__restrict__ l,
                 const uint32_t *__restrict__ fe) __attribute__((always_inline)) {
    constexpr bool kV = decltype(view)::value;
    if (mode == kSegGapSmall)
      seg_stream_body<kSegGapSmall, kU, kV>(lds, s_next, col, base, o, l, n, lg_chunk, fe, unit_raw, ev_h);
    else if (mode == kSegGapped)
      seg_stream_body<kSegGapped, kU, kV>(lds, s_next, col, base, o, l, n, lg_chunk, fe, unit_raw, ev_h);
    else if (mode == kSegPacked)
      seg_stream_body<kSegPacked, kU, kV>(lds, s_next, col, base, o, l, n, lg_chunk, fe, unit_raw, ev_h);
  };
  if (sorted) {
    seg_prof(14);
    run(std::true_type{}, ss.off, ss.len, ss.fev);
    seg_prof(15);
  } else {
    run(std::false_type{}, offs, lens, first_ev);
  }
}

__device__ __forceinline__ uint32_t seg_lds_tmul(const uint32_t *t, uint32_t v) {
  return xor3(t[v & 255u], t[256 + ((v >> 8) & 255u)], t[512 + ((v >> 16) & 255u)]) ^ t[768 + (v >> 24)];
}

// Per record [a, b) (events j and j+1), with U_x = x's unit, re_x = x's row
// end and H(x) = shift(raw(U_x .. x), re_x - x) from k_seg_stream:
//   shift(crc ^ ~0, re_b - b) = H(b) ^ shift(X, re_b - re_a),  X = H(a) ^ shift(~0, re_a - a)
// (raw(a||b) = shift(raw(a), |b|) ^ raw(b), and raw(W0) = ~0).  A record that
// starts and ends in one unit (70 % of config 5b's) shifts X by re_b - re_a
// <= 15 rows.  One that spans units carries X to its unit's end (<= 15 rows),
// chains the raw CRCs of the units it crosses (Horner, 16 rows per step) and
// shifts the result from U_b to re_b (1 .. 16 rows); no prefix over the whole
// span is needed (round 2 computed one with three scan kernels, 54 us at 2M
// records).  k_seg_plan caps records at kSegMaxRecord (1024 units).  Then one
// inverse shift by re_b - b in [1, 1024] bytes, by the octal digits of
// re_b - b - 1.  Every row shift is ONE table multiply (SegTables::rs) and the
// inverse shift four (SegTables::iv): 6 multiplies a record where the binary
// digits took 22 (round 3's first build, 38.6 us at 2M records), all tables in
// LDS (156 KiB, one workgroup per CU).  Waves work independently (persistent
// grid, no barrier after the table fill): an iteration of a wave covers kSub
// sub-passes of 64 events (H per lane) and 63 records (the end event's values
// from the next lane by a shuffle), every sub-pass's loads issued before the
// first is used.
template <uint32_t kU = kSegUnitLg>
__global__ __launch_bounds__(1024) void k_seg_combine(const uint8_t *base, const uint64_t *__restrict__ offs,
                                                      const uint32_t *__restrict__ lens, uint64_t n,
                                                      const uint32_t *__restrict__ flag,
                                                      const uint32_t *__restrict__ unit_raw,
                                                      const uint32_t *__restrict__ ev_h, uint32_t *__restrict__ crc_out,
                                                      const SegTables *__restrict__ st, uint32_t *__restrict__ taken,
                                                      uint32_t flags, const DeviceTables *__restrict__ tables,
                                                      const uint64_t *__restrict__ sorted_off,
                                                      const uint32_t *__restrict__ sorted_len,
                                                      const uint32_t *__restrict__ perm) {
  constexpr int kSub = 4, kIv0 = kSegRs * 1024;
  constexpr uint32_t kUnitRows = 1u << (kU - 10);
  __shared__ __attribute__((aligned(16))) uint32_t tl[(kSegRs + kSegIv) * 1024 + 256];
  const uint32_t mword = *flag;
  const bool sorted = (mword & kSegSortedBit) != 0;  // the stream ran over the sorted view (seg_sort)
  const uint32_t mode = mword & ~kSegSortedBit;
  if (taken && blockIdx.x == 0 && threadIdx.x == 0)  // (hc_debug_seg_taken: 1 packed, 2 gapped, 3 / 0 fallbacks; | 8 sorted)
    *taken = (mode == kSegPacked ? 1u : mode == kSegGapped ? 2u : mode == kSegFallbackGrp ? 3u : mode == kSegGapSmall ? 4u : 0u) |
             (sorted ? kSegSortedBit : 0u);
  // kSegFallbackGrp: k_crc_grp, launched after this kernel and gated on the
  // mode word, takes the batch.  (Round 5 first ran k_crc_grp's body here,
  // before the sweep: the plain fallback then read gridDim.x through an SGPR
  // pair hipcc wrote on the k_crc_grp path only -- an illegal address,
  // profiles/r5/r5d/, r6/fault/; the 34 ms on 1M aligned records was the plan's
  // O(n x units) fill of that build.)  Neither fallback needs
  // the SegTables below (r5: their fill was most of this kernel's 5 us then).
  if (mode == kSegFallbackGrp) return;
  if (mode == kSegFallback) {
    // the stream did not take the batch: k_crc_any's work over every message,
    // in this launch (round 3 launched k_crc_any after the combine, ~5 us a
    // call even when it exits at once); the body fills its own tables
    crc_any_body<true>(tl, base, offs, lens, 0, 0, flags, n, 0u, 0u, crc_out, nullptr, nullptr, tables, nullptr, 0);
    return;
  }
  {  // rs, iv and sh1 are contiguous in SegTables: every load issued before the first store
    static_assert(offsetof(SegTables, iv) == offsetof(SegTables, rs) + sizeof(SegTables::rs), "rs, iv adjacent");
    static_assert(offsetof(SegTables, sh1) == offsetof(SegTables, iv) + sizeof(SegTables::iv), "iv, sh1 adjacent");
    constexpr uint32_t kQ = (kSegRs + kSegIv) * 256 + 64, kPer = (kQ + 1023) / 1024;  // uint4s; per thread
    const uint4 *src = reinterpret_cast<const uint4 *>(&st->rs[0][0][0]);
    uint4 t[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t i = threadIdx.x + k * 1024u;
      t[k] = i < kQ ? src[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t i = threadIdx.x + k * 1024u;
      if (i < kQ) reinterpret_cast<uint4 *>(tl)[i] = t[k];
    }
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wv = (uint64_t)blockIdx.x * (blockDim.x >> 6) + uni(threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  auto rsh = [&](uint32_t v, uint32_t rows) {  // rows in [0, 16]
    return rows ? seg_lds_tmul(tl + (rows - 1u) * 1024u, v) : v;
  };
  auto inv_shift = [&](uint32_t y, uint32_t d) -> uint32_t {  // shift(y, -d), d in [1, 1024]: octal digits of d - 1
    const uint32_t e = d - 1u;
    const uint32_t *ti = tl + kIv0;
    y = seg_lds_tmul(ti + (e & 7u) * 1024u, y);
    if ((e >> 3) & 7u) y = seg_lds_tmul(ti + (kSegIvD1 - 1u + ((e >> 3) & 7u)) * 1024u, y);
    if ((e >> 6) & 7u) y = seg_lds_tmul(ti + (kSegIvD2 - 1u + ((e >> 6) & 7u)) * 1024u, y);
    if (e >> 9) y = seg_lds_tmul(ti + kSegIvD3 * 1024u, y);
    return y;
  };
  // the record [a, b), with x = offsets from A0 and H from the stream
  auto rec_crc = [&](uint64_t xa, uint32_t ha, uint64_t xb, uint32_t hb) -> uint32_t {
    const uint32_t re = (uint32_t)(xa >> 10) + 1u, rb = (uint32_t)(xb >> 10) + 1u;  // row ends, in rows from A0
    const uint32_t da = (uint32_t)(((uint64_t)re << 10) - xa), db = (uint32_t)(((uint64_t)rb << 10) - xb);
    const uint64_t ua = xa >> kU, ub = xb >> kU;
    const uint32_t X = ha ^ st->ones[da - 1];
    const uint32_t ue = (uint32_t)(ua + 1) * kUnitRows;  // a's unit end, in rows
    uint32_t v = rsh(X, ua < ub ? ue - re : rb - re);
    if (ua < ub) {  // the units a .. b-1 (Horner, 16 rows a step), then U_b -> re_b
      v ^= unit_raw[ua];
      for (uint64_t u = ua + 1; u < ub; u++) v = seg_lds_tmul(tl + (kUnitRows - 1u) * 1024u, v) ^ unit_raw[u];
      v = rsh(v, rb - (uint32_t)ub * kUnitRows);
    }
    return inv_shift(hb ^ v, db) ^ 0xFFFFFFFFu;
  };
  // the records of the stream's view: the batch's own arrays, or (sorted) the
  // sorted view's, record j's word going to batch entry perm[j].  Two
  // instantiations, not one with the arrays chosen at run time (whose
  // per-record perm select spilled VGPRs to scratch).
  auto records = [&](auto sorted_c, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens)
                     __attribute__((always_inline)) {
    constexpr bool kSorted = decltype(sorted_c)::value;
    const SegGeo geo = seg_geo<kU>(base, offs, lens, n);
    auto put = [&](uint64_t j, uint32_t v) { crc_out[kSorted ? perm[j] : j] = v; };
    if (mode == kSegGapSmall) {
      // record j = [s_j, e_j); the stream left H at s_0 (event 0) and at every
      // record end e_j (event j + 1) over the span's bytes, gaps included.  H(s_j)
      // from H(e_{j-1}): shifted by the rows between them, plus the gap bytes
      // [p, s_j) hashed here byte by byte (<= kSegSmallGap) and shifted to s_j's
      // row end; p = e_{j-1}, or s_j's unit start when the gap crosses into it
      // (then H(e_{j-1}) belongs to another unit and drops out).
      const uint32_t *sh1 = tl + (kSegRs + kSegIv) * 1024;
      for (uint64_t c = wv * 64u * kSub; c < n; c += nw * 64u * kSub) {
        uint64_t xa[kSub], xe[kSub];
        uint32_t ln[kSub], he[kSub], hb[kSub];
  #pragma unroll
        for (int p = 0; p < kSub; p++) {
          const uint64_t j = c + 64u * p + lane, jj = j < n ? j : n - 1, jp = jj ? jj - 1 : 0;
          xa[p] = (uint64_t)base + offs[jj] - geo.a0;
          ln[p] = lens[jj];
          xe[p] = (uint64_t)base + offs[jp] + lens[jp] - geo.a0;
          he[p] = ev_h[jj];
          hb[p] = ev_h[jj + 1];
        }
  #pragma unroll
        for (int p = 0; p < kSub; p++) {
          const uint64_t j = c + 64u * p + lane;
          const bool same = (xe[p] >> kU) == (xa[p] >> kU);
          const uint64_t gp = same ? xe[p] : (xa[p] >> kU) << kU;  // first gap byte in s_j's unit
          const uint32_t L = j < n && j ? (uint32_t)(xa[p] - gp) : 0u, nw = (L + 3u) >> 2;
          // before any lane leaves: a butterfly over a partial wave reads the
          // stale values of the lanes that left (r5l: a record after a 38-B gap
          // in wave 0, whose lane 0 holds record 0, lost its last words)
          const uint32_t nwmax = wave_max_u32(nw);
          if (j >= n) continue;
          uint32_t ha = he[p];  // j == 0: H(s_0) itself
          if (j) {
            // raw(gap bytes [gp, s_j)), L <= kSegSmallGap bytes, as nw words
            // ending at s_j behind 4nw - L leading zeros (raw ignores them).  The
            // words come from the aligned dwords D[i] at Bq + 4i, Bq = (s_j -
            // 4nw) & ~3, bytes before gp cleared, by a funnel shift of sa = s_j & 3
            // bytes.  Plain per-lane loads: a buffer resource is scalar, so one
            // built from a per-lane address became a 64-pass waterfall loop per
            // load (r5h/r5i: 233 / 369 us of combine at 2M records).  An aligned
            // dword holding a span byte never leaves the span's pages; D[nw] is
            // read only when it holds gap bytes (sa > 0).
            const uint32_t sa = (uint32_t)xa[p] & 3u;
            const uint64_t Bq = (xa[p] - 4u * nw) & ~3ull;
            uint32_t D[kSegSmallGap / 4 + 1];
            if (nwmax <= 5) {
              // gaps of <= 20 B (WAL headers: 17): the dwords from <= 3 aligned
              // 16-B loads, C0 = the chunk holding the first dword with gap bytes,
              // a chunk loaded only when it holds a dword the loop below reads
              // (six dword loads a record took 98.6 us of combine at 2M records,
              // these 82.8: the gap reads are bound by their instruction count,
              // profiles/r6/r6u/)
              const uint64_t i0 = gp > Bq ? (gp - Bq) >> 2 : 0;  // first dword with gap bytes
              const uint64_t a0w = Bq + 4u * i0, C0 = a0w & ~15ull;
              const uint32_t ilast = sa ? nw : nw - 1;             // last dword read
              const uint64_t alast = Bq + 4u * ilast;
              uint32_t Q[12];
  #pragma unroll
              for (int k = 0; k < 3; k++) {
                const uint64_t ck = C0 + 16u * k;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (nw && ck <= alast) v = *reinterpret_cast<const uint4 *>(geo.a0 + ck);
                Q[4 * k] = v.x; Q[4 * k + 1] = v.y; Q[4 * k + 2] = v.z; Q[4 * k + 3] = v.w;
              }
  #pragma unroll
              for (uint32_t i = 0; i <= kSegSmallGap / 4; i++) {
                D[i] = 0;
                if (i > 5) continue;
                const uint64_t ai = Bq + 4u * i;
                if (i <= nw && ai + 4u > gp && (i < nw || sa)) {
                  const uint32_t qi = (uint32_t)(((int64_t)ai - (int64_t)C0) >> 2);
                  uint32_t v = 0;
  #pragma unroll
                  for (uint32_t t = 0; t < 12; t++) v = qi == t ? Q[t] : v;
                  D[i] = v;
                  if (ai < gp) D[i] &= ~0u << (8u * (uint32_t)(gp - ai));
                }
              }
            } else {
  #pragma unroll
              for (uint32_t i = 0; i <= kSegSmallGap / 4; i++) {
                D[i] = 0;
                if (i > nwmax) continue;
                const uint64_t ai = Bq + 4u * i;
                if (i <= nw && ai + 4u > gp && (i < nw || sa)) {
                  D[i] = *reinterpret_cast<const uint32_t *>(geo.a0 + ai);
                  if (ai < gp) D[i] &= ~0u << (8u * (uint32_t)(gp - ai));
                }
              }
            }
            uint32_t r = 0;
  #pragma unroll
            for (uint32_t k = 0; k < kSegSmallGap / 4; k++) {
              if (k >= nwmax) break;
              uint32_t t = r, w = __builtin_amdgcn_alignbyte(D[k + 1], D[k], sa);
  #pragma unroll
              for (int q = 0; q < 4; q++) {
                t = sh1[(t ^ w) & 255u] ^ (t >> 8);
                w >>= 8;
              }
              r = k < nw ? t : r;
            }
            const uint32_t re = (uint32_t)(xa[p] >> 10) + 1u, d = (uint32_t)(((uint64_t)re << 10) - xa[p]);
            // shift(r, d) = shift(shift(r, 1024), -(1024 - d))
            uint32_t pg = seg_lds_tmul(tl, r);
            if (d < 1024u) pg = inv_shift(pg, 1024u - d);
            ha = (same ? rsh(he[p], (uint32_t)((xa[p] >> 10) - (xe[p] >> 10))) : 0u) ^ pg;
          }
          put(j, rec_crc(xa[p], ha, xa[p] + ln[p], hb[p]));
        }
      }
      return;
    }
    if (mode == kSegGapped) {
      // record j = [s_j, e_j), events 2j and 2j+1, one record a lane.  The
      // stream zeroed the gap bytes and left H at e_j (2j+1) and s_0 (0): H(s_j)
      // is H(e_{j-1}) shifted by the rows between them in one unit, else 0
      // (k_seg_stream's kGap notes)
      for (uint64_t c = wv * 64u * kSub; c < n; c += nw * 64u * kSub) {
        uint64_t xa[kSub], xe[kSub];
        uint32_t ln[kSub], he[kSub], hb[kSub];
  #pragma unroll
        for (int p = 0; p < kSub; p++) {
          const uint64_t j = c + 64u * p + lane, jj = j < n ? j : n - 1, jp = jj ? jj - 1 : 0;
          xa[p] = (uint64_t)base + offs[jj] - geo.a0;
          ln[p] = lens[jj];
          xe[p] = (uint64_t)base + offs[jp] + lens[jp] - geo.a0;
          he[p] = ev_h[jj ? 2 * jj - 1 : 0];
          hb[p] = ev_h[2 * jj + 1];
        }
  #pragma unroll
        for (int p = 0; p < kSub; p++) {
          const uint64_t j = c + 64u * p + lane;
          uint32_t ha = he[p];  // j == 0: H(s_0) itself
          if (j) ha = (xe[p] >> kU) == (xa[p] >> kU) ? rsh(he[p], (uint32_t)((xa[p] >> 10) - (xe[p] >> 10))) : 0u;
          if (j < n) put(j, rec_crc(xa[p], ha, xa[p] + ln[p], hb[p]));
        }
      }
      return;
    }
    for (uint64_t c = wv * 63u * kSub; c < n; c += nw * 63u * kSub) {
      uint64_t x[kSub];
      uint32_t eh[kSub];
  #pragma unroll
      for (int p = 0; p < kSub; p++) {  // event c + 63p + lane (past n: the span's end again)
        const uint64_t j = c + 63u * p + lane, jj = j < n ? j : n;
        x[p] = (jj < n ? (uint64_t)base + offs[jj] : geo.pend) - geo.a0;
        eh[p] = ev_h[jj];
      }
  #pragma unroll
      for (int p = 0; p < kSub; p++) {
        const uint64_t j = c + 63u * p + lane;
        const uint32_t kb = __shfl_down(eh[p], 1);
        const uint64_t xb = __shfl_down((unsigned long long)x[p], 1);
        if (lane < 63 && j < n) put(j, rec_crc(x[p], eh[p], xb, kb));
      }
    }
  };
  if (sorted)
    records(std::true_type{}, sorted_off, sorted_len);
  else
    records(std::false_type{}, offs, lens);
}

// A uniform block batch k_crc_grp refuses, on the message stream
// (launch_seg_blocks): its messages block[hdr:ulen] as off/len arrays (hdr 4:
// the payload after the stored word; 0: a uniform whole-message batch) ...
__global__ __launch_bounds__(256) void k_seg_block_msgs(uint64_t n, uint64_t stride, uint32_t ulen, uint32_t hdr,
                                                        uint64_t *__restrict__ moff, uint32_t *__restrict__ mlen) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    moff[j] = j * stride + hdr;
    mlen[j] = ulen - hdr;
  }
}

// ... and the blocks' outputs from the message CRCs: CheckBlockIntegrity's
// compare (crc_util.go:88-100) into the bitmap and first_bad, then
// AddCRCToBlockData's store (:21-33), as k_crc_any does them (the stored word
// read before the stamp).  A wave takes 64 consecutive blocks: one bitmap
// atomic per 32 with a bad block, one first_bad lowering per wave.
__global__ __launch_bounds__(256) void k_seg_block_out(const uint8_t *base, uint64_t n, uint64_t stride,
                                                       uint32_t flags, const uint32_t *__restrict__ crcs,
                                                       uint32_t *__restrict__ bad_bitmap,
                                                       unsigned long long *__restrict__ first_bad) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  // The route exists for blocks k_crc_grp refuses, often at addresses that are
  // not 4-B aligned: then the stored word is read and written bytewise (ADVICE
  // r5: a misaligned u32 access is UB the compiler may lower assuming alignment)
  const bool al4 = (((uintptr_t)base | stride) & 3u) == 0;  // kernel-uniform
  auto get32 = [&](const uint8_t *q) -> uint32_t {
    if (al4) return *reinterpret_cast<const uint32_t *>(q);
    return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  };
  auto put32 = [&](uint8_t *q, uint32_t v) {  // PutUint32LE
    if (al4) {
      *reinterpret_cast<uint32_t *>(q) = v;
    } else {
      q[0] = (uint8_t)v;
      q[1] = (uint8_t)(v >> 8);
      q[2] = (uint8_t)(v >> 16);
      q[3] = (uint8_t)(v >> 24);
    }
  };
  for (uint64_t c = w0 * 64u; c < n; c += nw * 64u) {
    const uint64_t j = c + lane;
    const bool in = j < n;
    uint8_t *p = const_cast<uint8_t *>(base) + (in ? j : 0) * stride;
    const uint32_t crc = in ? crcs[j] : 0u;
    if (first_bad) {
      const uint32_t stored = in ? get32(p) : 0u;
      const uint64_t bad = __ballot(in && stored != crc);
      if (bad) {  // wave-uniform
        if (bad_bitmap && lane == 0 && (uint32_t)bad) atomicOr(bad_bitmap + (c >> 5), (uint32_t)bad);
        if (bad_bitmap && lane == 32 && (bad >> 32)) atomicOr(bad_bitmap + (c >> 5) + 1, (uint32_t)(bad >> 32));
        if (lane == 0) atomicMin(first_bad, (unsigned long long)(c + (uint64_t)__builtin_ctzll(bad)));
      }
    }
    if (in && (flags & kFlagStamp)) put32(p, crc);
  }
}

}  // namespace

// uniform batches of 16-B aligned 1 KiB-multiple blocks (k_crc_fast)
hipError_t launch_fast(const Batch &b, int grid, hipStream_t s) {
  if (!b.base || b.off || b.len || b.ulen == 0 || (b.ulen & 1023u) != 0 || (b.stride & 15u) != 0 ||
      (reinterpret_cast<uintptr_t>(b.base) & 15u) != 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_crc_fast, dim3(grid), dim3(kFastThreads), 0, s, b.base, b.stride, b.ulen, b.flags, b.nblocks,
                     b.crc_out, b.bad_bitmap, b.first_bad, b.tables);
  return hipGetLastError();
}

// k_crc_any: 64-message windows handed out one at a time (tools/kbench2,
// profiles/r2/any/: 2M records, config 5b +4.5 %, equal 9815-B records
// +2.7 %, 4092-B blocks +2 % over static runs per wave).  Whole-message
// batches hash their records of <= 1020 bytes lane-parallel (1.77x on small
// records, neutral on config 5b and on large ones, profiles/r2/any_small_lanes/);
// block mode keeps the leaner build.
hipError_t launch_general(const Batch &b, uint32_t fast_mask, int grid, hipStream_t s) {
  if (!b.base) return hipErrorInvalidValue;
  if (b.flags & kFlagMessages)
    hipLaunchKernelGGL(k_crc_any<true>, dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, b.stride, b.ulen,
                       b.flags, b.nblocks, fast_mask, 0u, b.crc_out, b.bad_bitmap, b.first_bad, b.tables, b.skip_slot,
                       b.skip_tag);
  else
    hipLaunchKernelGGL(k_crc_any<false>, dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, b.stride, b.ulen,
                       b.flags, b.nblocks, fast_mask, 0u, b.crc_out, b.bad_bitmap, b.first_bad, b.tables, b.skip_slot,
                       b.skip_tag);
  return hipGetLastError();
}

// XCD-contiguous chunk slots: 8/16 KiB uniform batches up to 4M blocks (1M
// blocks: +0.3-0.9 % on four boxes; 16M blocks: -0.3-0.7 %, workgroup order
// at C = 128 kept there; profiles/r2/ab_xcd/)
bool grp_xcd(uint32_t block_bytes, int grid, uint64_t nblocks) {
  return block_bytes >= 8192 && (grid & 7) == 0 && nblocks <= (4ull << 20);
}

uint32_t grp_lg_chunk(uint64_t nblocks, int grid, uint32_t block_bytes) {
  // Chunk of C = 2^lg consecutive blocks per workgroup (tools/kbench2 sweeps,
  // profiles/r2/sweep*: 1M blocks, C = 8 .. 512, four boxes): 4 KiB blocks at
  // C = 64 (84-85 % of 8 TB/s), mixed 4/8/16 KiB off/len batches (block_bytes
  // 0) at C = 32-64.  8 and 16 KiB blocks with the XCD-contiguous slot order
  // (grp_xcd; profiles/r2/ab_xcd/, three boxes) at C = 32 and 16: +0.3-0.9 %
  // over C = 128 in workgroup order.  Small batches keep at least 4 chunks per
  // workgroup.  HC_LG_CHUNK overrides (tuning sweeps only).
  static const int forced = env_int("HC_LG_CHUNK", -1);
  uint32_t lg = forced >= 0                             ? (uint32_t)forced
                : !grp_xcd(block_bytes, grid, nblocks)  ? (block_bytes >= 8192 ? 7u : 6u)
                : block_bytes >= 16384                  ? 4u
                                                        : 5u;
  if (forced < 0)
    while (lg > 0 && (nblocks >> lg) < (uint64_t)grid * 4) lg--;
  return lg;
}

hipError_t launch_grp(const Batch &b, int grid, hipStream_t s) {
  // layout contract: uniform batches of 16-B aligned 4 KiB-multiple blocks, or
  // both off and len arrays (non-conforming entries are skipped on the device)
  if (!b.base || (!b.off != !b.len)) return hipErrorInvalidValue;
  if (!b.off && (b.ulen == 0 || (b.ulen & 4095u) != 0 || (b.stride & 15u) != 0 ||
                 (reinterpret_cast<uintptr_t>(b.base) & 15u) != 0))
    return hipErrorInvalidValue;
  const uint32_t lg = grp_lg_chunk(b.nblocks, grid, (b.off || b.len) ? 0u : b.ulen);
  if (b.off || b.len)
    hipLaunchKernelGGL((k_crc_grp<true>), dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, b.stride,
                       b.ulen, b.flags, b.nblocks, lg, b.crc_out, b.bad_bitmap, b.first_bad, b.tables, b.skip_slot,
                       b.skip_tag);
  else if (grp_xcd(b.ulen, grid, b.nblocks))  // each XCD's workgroups own neighbouring chunk slots
    hipLaunchKernelGGL((k_crc_grp<false, true>), dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, b.stride,
                       b.ulen, b.flags, b.nblocks, lg, b.crc_out, b.bad_bitmap, b.first_bad, b.tables);
  else
    hipLaunchKernelGGL((k_crc_grp<false>), dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, b.stride,
                       b.ulen, b.flags, b.nblocks, lg, b.crc_out, b.bad_bitmap, b.first_bad, b.tables);
  return hipGetLastError();
}

hipError_t launch_frame(const uint8_t *src, uint64_t n, uint8_t *dst, uint32_t *crc_out,
                        const DeviceTables *tables, int grid, hipStream_t s) {
  const uint64_t nblk = (n + 4091) / 4092;
  if (nblk == 0) return hipSuccess;
  // workgroup 0: the two edge blocks; then one interior block per wave, in
  // runs of 4 x kFrameSpread blocks over kFrameSpread workgroups
  const uint64_t wgs = 1 + (nblk > 2 ? kFrameSpread * ((nblk - 2 + 4 * kFrameSpread - 1) / (4 * kFrameSpread)) : 0);
  if (wgs > kMaxGridWgs) return hipErrorInvalidValue;  // gridDim.x * 256 must stay below 2^32
  hipLaunchKernelGGL(k_frame, dim3((unsigned)wgs), dim3(256), 0, s, src, n, dst, nblk, crc_out, tables);
  return hipGetLastError();
}

hipError_t launch_unframe(const uint8_t *blocks, uint64_t nblk, uint32_t lg_groups, uint8_t *out,
                          uint32_t *crc_out, uint32_t *bad_bitmap, unsigned long long *first_bad,
                          const DeviceTables *tables, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  if (!blocks || !out || lg_groups > 2) return hipErrorInvalidValue;
  const uint64_t grid = unframe_grid(nblk, lg_groups);  // one 4 KiB group per wave, 4 waves per workgroup
  if (grid > kMaxGridWgs) return hipErrorInvalidValue;  // gridDim.x * 256 must stay below 2^32
#define HC_UNFRAME(L)                                                                                      \
  hipLaunchKernelGGL((k_unframe<L>), dim3((unsigned)grid), dim3(256), 0, s, blocks, nblk, out, crc_out, bad_bitmap, \
                     first_bad, tables)
  if (lg_groups == 0)
    HC_UNFRAME(0);
  else if (lg_groups == 1)
    HC_UNFRAME(1);
  else
    HC_UNFRAME(2);
#undef HC_UNFRAME
  return hipGetLastError();
}

hipError_t launch_fill(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                       uint32_t ulen, uint64_t n, uint64_t seed, int grid, hipStream_t s, uint64_t first) {
  hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, s, base, off, len, stride, ulen, n, seed, first);
  return hipGetLastError();
}

uint64_t seg_max_units(uint64_t span_bound) { return (span_bound >> kSegUnitLg) + 2; }

hipError_t seg_prof_read(uint64_t *out16) {
  return hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_seg_prof), sizeof(g_seg_prof), 0, hipMemcpyDeviceToHost);
}

uint64_t seg_workspace_bytes(uint64_t n, uint64_t max_units, bool sort) {
  return seg_ws_layout(nullptr, n, max_units, sort).bytes;
}

hipError_t launch_seg(const Batch &b, const SegTables *st, uint32_t *ws, uint64_t max_units, int grid, hipStream_t s,
                      uint32_t *taken, uint64_t grp_min, uint64_t sort_min, uint32_t sync_spins, uint32_t sort_uc,
                      uint32_t lg_chunk) {
  if (!b.base || !b.off || !b.len || !b.crc_out || !st || !ws || b.nblocks == 0 || !(b.flags & kFlagMessages))
    return hipErrorInvalidValue;
  const uint64_t n = b.nblocks;
  // the sorted view (seg_sort): from sort_min records, on a grid it can meet at barriers
  const bool sort = sort_min && n >= sort_min && grid <= (int)kSegSortMaxWgs;
  const SegWs w = seg_ws_layout(ws, n, max_units, sort);
  const uint64_t pg = (n + 256) / 256;
  // HC_SEG_PLAN_WGS overrides the plan's grid cap, up to kSegPlanMaxWgs (tuning sweeps)
  static const uint64_t cap = (uint64_t)std::max(1, std::min((int)kSegPlanMaxWgs, env_int("HC_SEG_PLAN_WGS", (int)kSegPlanWgs)));
  const uint32_t plan_wgs = (uint32_t)(pg < cap ? pg : cap);
  // every launch checked: a later kernel must not run on a failed one's stale
  // outputs (hipGetLastError reports the latest call, not the first failure)
  hipLaunchKernelGGL(k_seg_plan<>, dim3(plan_wgs), dim3(256), 0, s, b.base, b.off, b.len, n, max_units, w.plan_bad,
                     w.plan_gx, w.plan_conf, w.first_ev, w.ss.sync);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // a batch large enough that a gated launch (exiting on its first load unless
  // the stream chose kSegFallbackGrp: 5 us under rocprofv3, r5e) is small against it
  // (grp_min: HC_SEG_GRP_MIN, default kSegGrpFallbackMin)
  const uint32_t allow_grp = n >= grp_min ? 1u : 0u;
  hipLaunchKernelGGL(k_seg_stream<>, dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, n, lg_chunk,
                     w.plan_bad, w.plan_gx, w.plan_conf, plan_wgs, allow_grp, w.flag, w.first_ev, w.unit_raw, w.ev_h,
                     b.tables, max_units, ws, sort ? 1u : 0u, sync_spins, sort_uc);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_seg_combine<>, dim3(grid), dim3(1024), 0, s, b.base, b.off, b.len, n, w.flag, w.unit_raw,
                     w.ev_h, b.crc_out, st, taken, b.flags, b.tables, w.ss.off, w.ss.len, w.ss.perm);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (allow_grp)
    hipLaunchKernelGGL((k_crc_grp<true>), dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, b.stride, b.ulen,
                       b.flags, n, grp_lg_chunk(n, grid, 0), b.crc_out, nullptr, nullptr, b.tables, nullptr, 0,
                       w.flag);
  return hipGetLastError();
}

uint64_t seg_block_workspace_bytes(uint64_t n, uint64_t max_units, bool crc_words) {
  return ((seg_workspace_bytes(n, max_units) + 7) & ~7ull) + 12 * n + (crc_words ? 4 * n : 0);
}

hipError_t launch_seg_blocks(const Batch &b, const SegTables *st, uint32_t *ws, uint64_t max_units, int grid,
                             hipStream_t s, uint32_t *taken) {
  const uint64_t n = b.nblocks;
  // whole-message mode (a uniform HC_F_MESSAGES batch): the messages are the
  // strided entries themselves, and crc_out is their only output (k_crc_any
  // neither verifies nor stamps messages)
  const bool msg = (b.flags & kFlagMessages) != 0;
  if (!b.base || b.off || b.len || b.ulen < 4 || b.stride < b.ulen || !st || !ws || n == 0 || !b.tables ||
      (msg && !b.crc_out))
    return hipErrorInvalidValue;
  uint64_t *moff = reinterpret_cast<uint64_t *>(ws + ((seg_workspace_bytes(n, max_units) + 7) & ~7ull) / 4);
  uint32_t *mlen = reinterpret_cast<uint32_t *>(moff + n), *wcrc = mlen + n;
  const int mg = (int)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_seg_block_msgs, dim3(mg), dim3(256), 0, s, n, b.stride, b.ulen, msg ? 0u : 4u, moff, mlen);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  Batch mb = b;
  mb.off = moff;
  mb.len = mlen;
  mb.flags = kFlagMessages;
  mb.crc_out = b.crc_out ? b.crc_out : wcrc;
  mb.bad_bitmap = nullptr;
  mb.first_bad = nullptr;
  // no k_crc_grp fallback: these blocks are not its shape, and its fallback would hash whole messages
  if ((e = launch_seg(mb, st, ws, max_units, grid, s, taken, ~0ull)) != hipSuccess) return e;
  if (msg || (!b.first_bad && !(b.flags & kFlagStamp))) return hipSuccess;
  hipLaunchKernelGGL(k_seg_block_out, dim3(mg), dim3(256), 0, s, b.base, n, b.stride, b.flags, mb.crc_out,
                     b.bad_bitmap, b.first_bad);
  return hipGetLastError();
}

hipError_t launch_verify_prepare(uint32_t *bitmap, unsigned long long *first_bad, uint64_t n,
                                 hipStream_t s) {
  const uint64_t words = (n + 31) / 32;
  int grid = (int)((words + 255) / 256);
  if (grid < 1) grid = 1;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(k_verify_prepare, dim3(grid), dim3(256), 0, s, bitmap, first_bad, words);
  return hipGetLastError();
}

}  // namespace hc
