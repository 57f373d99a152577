// r1_kernels.hip -- the round-1 production kernel k_crc_uni (uniform 4/8/16 KiB
// blocks, static interleaved block order), kept OUT of the product as the
// baseline of the A/B harnesses (tools/kbench*.hip include it after
// hunddb_amd/csrc/hc_kernels.hip).  Replaced in the product by k_crc_grp
// (per-CU chunked dynamic hand-out).
namespace hc {
namespace {
// k_crc_uni: the streaming kernel specialised for uniform batches whose block
// length is a multiple of 4 KiB (every on-disk block size: 4/8/16 KiB).  A
// block is ulen/4096 groups of four 1 KiB rows; the wave's four row registers
// always hold one group, so a row's slot, its block and its place in the block
// are static and the producer is one scalar pointer per group (the next
// group's rows are loads at immediate offsets 0/1K/2K/3K of one address).
// Block order is interleaved (block b -> wave b mod W).  Same tables, Horner
// streams, lane placement and lane-0 side effects as k_crc_fast.
template <int kWaves, bool kNull = false>
__global__ __launch_bounds__(kWaves * 64) void k_crc_uni(const uint8_t *base, uint64_t stride, uint32_t ulen,
                                                        uint32_t flags, uint64_t nblocks,
                                                        uint32_t *__restrict__ crc_out,
                                                        uint32_t *__restrict__ bad_bitmap,
                                                        unsigned long long *__restrict__ first_bad,
                                                        const DeviceTables *__restrict__ tables) {
  constexpr int kThreads = kWaves * 64;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  // table image: identical to k_crc_fast's (4 s4 replicas)
  const uint32_t *tg = &tables->tg[0][0];
  for (uint32_t q = tid; q < kLdsMainBytes / 16; q += kThreads) {
    const uint32_t a = q * 16;
    const uint32_t k = ((a >> 16) << 1) | ((a >> 7) & 1u);
    const uint32_t v = tg[k * 256 + ((a >> 8) & 255u)];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + a) = make_uint4(v, v, v, v);
  }
  const uint32_t *s4 = &tables->s4[0][0];
  for (uint32_t q = tid; q < kLdsS4Bytes / 16; q += kThreads) {
    const uint32_t v = s4[q];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + kLdsMainBytes + q * 16) = make_uint4(v, v, v, v);
  }
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  const uint32_t w0 = tables->w0;
  __syncthreads();

  const uint32_t r4 = (lane & 31u) << 2;
  const uint32_t B0 = r4, B1 = r4 | 128u, B2 = 65536u | r4, B3 = 65536u | 128u | r4;
  const uint32_t S4base = kLdsMainBytes + ((lane & 3u) << 2);
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    if constexpr (kNull) return c ^ w;
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
  const uint64_t W = (uint64_t)gridDim.x * kWaves;
  uint64_t b = (uint64_t)blockIdx.x * kWaves + wave;
  if (b >= nblocks) return;
  const uint32_t groups = ulen >> 12;
  const bool msg = (flags & kFlagMessages) != 0;
  const uint8_t *gp = base + b * stride;  // the group the row registers hold
  uint4 q0 = load_row<1>(gp, lane), q1 = load_row<1>(gp + 1024, lane), q2 = load_row<1>(gp + 2048, lane),
        q3 = load_row<1>(gp + 3072, lane);
  uint32_t g = 0, c0 = 0, c1 = 0, c2 = 0, c3 = 0, stored = 0;
  bool reported = false;  // wave-uniform: this wave already lowered first_bad (see k_crc_fast)
  for (;;) {
    // next group: the block's next 4 rows, or the first 4 rows of the wave's
    // next block (past the last block: this group again, never consumed)
    const uint32_t ng = g + 1 == groups ? 0u : g + 1;
    const uint64_t nb = ng ? b : b + W;
    const uint8_t *np = ng ? gp + 4096 : (nb < nblocks ? base + nb * stride : gp);
    // each row register is refilled right after its row is hashed (same
    // registers across iterations: no copies, no drain at the loop latch)
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
    q0 = load_row<1>(np, lane);
    c0 = row_step(c0, q1.x);
    c1 = row_step(c1, q1.y);
    c2 = row_step(c2, q1.z);
    c3 = row_step(c3, q1.w);
    q1 = load_row<1>(np + 1024, lane);
    c0 = row_step(c0, q2.x);
    c1 = row_step(c1, q2.y);
    c2 = row_step(c2, q2.z);
    c3 = row_step(c3, q2.w);
    q2 = load_row<1>(np + 2048, lane);
    c0 = row_step(c0, q3.x);
    c1 = row_step(c1, q3.y);
    c2 = row_step(c2, q3.z);
    c3 = row_step(c3, q3.w);
    q3 = load_row<1>(np + 3072, lane);
    if (ng == 0) {  // block b is complete
      uint32_t crc;
      if constexpr (kNull) {
        crc = wave_xor(c0 ^ c1 ^ c2 ^ c3);
      } else {
        const uint32_t d = shift4(shift4(shift4(c0, c1), c2), c3);
        crc = wave_xor(matvec32(col, d)) ^ 0xFFFFFFFFu;
      }
      const uint8_t *bp = base + b * stride;
      if (crc_out) lane0_store_u32(crc_out + b, crc);
      if (flags & kFlagStamp) lane0_store_u32(const_cast<uint32_t *>(reinterpret_cast<const uint32_t *>(bp)), crc);
      const bool bad = uni(stored) != crc;
      if (first_bad && bad) {
        if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
        if (!reported) lane0_atomic_umin64(first_bad, b);
        reported = true;
      }
      if (nb >= nblocks) return;
      b = nb;
    }
    g = ng;
    gp = np;
  }
}

}  // namespace

hipError_t launch_uni(const Batch &b, int grid, hipStream_t s) {
  if (b.ulen == 0 || (b.ulen & 4095u) != 0 || !b.base) return hipErrorInvalidValue;  // its layout contract
  hipLaunchKernelGGL((k_crc_uni<kFastWaves>), dim3(grid), dim3(kFastThreads), 0, s, b.base, b.stride, b.ulen, b.flags,
                     b.nblocks, b.crc_out, b.bad_bitmap, b.first_bad, b.tables);
  return hipGetLastError();
}

}  // namespace hc
