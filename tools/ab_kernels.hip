// ab_kernels.hip -- A/B kernels measured in round 2 and kept OUT of the product
// (tools/kbench2.hip and tools/kframe.hip include this file after
// ab_hc_kernels.hip (the round-2 product source), in the same namespace, so they reuse its
// helpers).  Results: DESIGN.md section 4.1a (k_crc_piece, not kept: +0-0.5 %)
// and section 4.4a (k_frame_np, not kept: 8-37 % slower).
namespace hc {
namespace {

// ---------------------------------------------------------------------------
// k_crc_piece: uniform batches of G x 4 KiB blocks (G = 2, 4) handed out by
// 4 KiB pieces instead of whole blocks.  A read stream with k_crc_grp's
// hand-out reads 1-2 % faster with 4 KiB pieces than with 8 KiB ones
// (tools/kread, profiles/r2/read_ceiling/).  A wave hashes its piece like a
// 4 KiB block (lane 0's first word of piece 0 replaced by W0) and finalises it
// to R_g = raw(piece g); the block's raw CRC is XOR_g shift(R_g, 4096 (G-1-g))
// (raw(a||b) = shift(raw(a), |b|) ^ raw(b)).  The pieces' shifted values meet
// in an LDS slot of the block (XOR + arrival mask, slot = the block's hand-out
// sequence number mod kPieceSlots); the last piece to arrive stores the CRC,
// stamps, verifies.  Shift tables: SegTables::pw[2] (4096 B), pw[3] (8192 B).
constexpr uint32_t kPieceSlots = 256;
template <int G, bool kXcd = false>
__global__ __launch_bounds__(kFastThreads) void k_crc_piece(const uint8_t *base, uint64_t stride, uint32_t flags,
                                                           uint64_t nblocks, uint32_t lg_chunk,
                                                           uint32_t *__restrict__ crc_out,
                                                           uint32_t *__restrict__ bad_bitmap,
                                                           unsigned long long *__restrict__ first_bad,
                                                           const DeviceTables *__restrict__ tables,
                                                           const SegTables *__restrict__ st) {
  static_assert(G == 2 || G == 4, "pieces per block");
  constexpr uint32_t kLgG = G == 2 ? 1u : 2u, kFull = (1u << G) - 1u;
  constexpr int kShT = G == 2 ? 1 : 2;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4];
  __shared__ uint32_t tsh[kShT * 1024];
  __shared__ uint32_t s_acc[kPieceSlots], s_mask[kPieceSlots], s_stored[kPieceSlots];
  __shared__ uint32_t s_next;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t *tg = &tables->tg[0][0];
  for (uint32_t q = tid; q < kLdsMainBytes / 16; q += kFastThreads) {
    const uint32_t a = q * 16;
    const uint32_t k = ((a >> 16) << 1) | ((a >> 7) & 1u);
    const uint32_t v = tg[k * 256 + ((a >> 8) & 255u)];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + a) = make_uint4(v, v, v, v);
  }
  const uint32_t *s4 = &tables->s4[0][0];
  for (uint32_t q = tid; q < kLdsS4Bytes / 16; q += kFastThreads) {
    const uint32_t v = s4[q];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + kLdsMainBytes + q * 16) = make_uint4(v, v, v, v);
  }
  for (uint32_t q = tid; q < kShT * 1024u; q += kFastThreads) tsh[q] = (&st->pw[2][0][0])[q];
  for (uint32_t q = tid; q < kPieceSlots; q += kFastThreads) {
    s_acc[q] = 0;
    s_mask[q] = 0;
  }
  if (tid == 0) s_next = 3 * kFastWaves;  // hand-out indices 0 .. 3W-1 are dealt statically below
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
  auto tmul = [&](const uint32_t *t, uint32_t v) -> uint32_t {  // v wave-uniform: broadcast reads
    return xor3(xor3(t[v & 255u], t[256 + ((v >> 8) & 255u)], t[512 + ((v >> 16) & 255u)]), t[768 + (v >> 24)], 0u);
  };

  const uint32_t wave = uni(tid >> 6);
  const uint64_t Gg = gridDim.x;
  const uint64_t wg = kXcd && (Gg & 7u) == 0 ? (blockIdx.x & 7u) * (Gg >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const uint32_t cmask = (1u << lg_chunk) - 1u;  // lg_chunk >= kLgG: a chunk holds whole blocks
  auto pc_of = [&](uint32_t k) -> uint64_t { return (((uint64_t)(k >> lg_chunk) * Gg + wg) << lg_chunk) | (k & cmask); };
  const uint64_t np_ = nblocks << kLgG;
  auto pa = [&](uint64_t p) -> const uint8_t * {
    return base + (p >> kLgG) * stride + ((uint32_t)p & (G - 1u)) * 4096u;
  };

  uint32_t kc = wave, k1 = kFastWaves + wave, k2 = 2 * kFastWaves + wave;
  uint64_t pc = pc_of(kc);
  if (pc >= np_) return;
  uint64_t p1 = pc_of(k1), p2 = pc_of(k2);
  const uint8_t *gp = pa(pc);
  uint4 q0 = load_row<1>(gp, lane), q1 = load_row<1>(gp + 1024, lane), q2 = load_row<1>(gp + 2048, lane),
        q3 = load_row<1>(gp + 3072, lane);
  uint32_t k3v = 0;  // VGPR: the LDS hand-out result, read one piece later
  if (lane == 0) k3v = atomicAdd(&s_next, 1u);
  uint64_t reported = ~0ull;
  for (;;) {
    const bool nv = p1 < np_;
    const uint8_t *npa = nv ? pa(p1) : gp;  // past the end: re-read this piece, never consumed
    const uint32_t g = (uint32_t)pc & (G - 1u);
    uint4 v = q0;
    uint32_t stored = 0;
    if (lane == 0 && g == 0) {
      stored = v.x;
      v.x = w0;
    }
    uint32_t c0 = v.x, c1 = v.y, c2 = v.z, c3 = v.w;
    q0 = load_row<1>(npa, lane);
    __builtin_amdgcn_sched_barrier(0);
    c0 = row_step(c0, q1.x);
    c1 = row_step(c1, q1.y);
    c2 = row_step(c2, q1.z);
    c3 = row_step(c3, q1.w);
    __builtin_amdgcn_sched_barrier(0);
    q1 = load_row<1>(npa + 1024, lane);
    __builtin_amdgcn_sched_barrier(0);
    c0 = row_step(c0, q2.x);
    c1 = row_step(c1, q2.y);
    c2 = row_step(c2, q2.z);
    c3 = row_step(c3, q2.w);
    __builtin_amdgcn_sched_barrier(0);
    q2 = load_row<1>(npa + 2048, lane);
    __builtin_amdgcn_sched_barrier(0);
    c0 = row_step(c0, q3.x);
    c1 = row_step(c1, q3.y);
    c2 = row_step(c2, q3.z);
    c3 = row_step(c3, q3.w);
    __builtin_amdgcn_sched_barrier(0);
    q3 = load_row<1>(npa + 3072, lane);
    __builtin_amdgcn_sched_barrier(0);
    // the piece's raw CRC, placed at the block end
    const uint32_t d = shift4(shift4(shift4(c0, c1), c2), c3);
    uint32_t r = wave_xor(matvec32(col, d));
    if constexpr (G == 2) {
      if (g == 0) r = tmul(tsh, r);
    } else {
      if ((3u - g) & 1u) r = tmul(tsh, r);
      if ((3u - g) & 2u) r = tmul(tsh + 1024, r);
    }
    // meet the block's other pieces in its slot; the last one finishes the block
    const uint32_t slot = (kc >> kLgG) & (kPieceSlots - 1u);
    uint32_t prev = 0;
    if (lane == 0) {
      if (g == 0) __hip_atomic_store(&s_stored[slot], stored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_xor(&s_acc[slot], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      prev = __hip_atomic_fetch_or(&s_mask[slot], 1u << g, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if ((uni(prev) | (1u << g)) == kFull) {  // wave-uniform
      uint32_t raw = 0, sw = 0;
      if (lane == 0) {
        raw = __hip_atomic_load(&s_acc[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        sw = __hip_atomic_load(&s_stored[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&s_acc[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&s_mask[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      const uint32_t crc = uni(raw) ^ 0xFFFFFFFFu;
      const uint64_t b = pc >> kLgG;
      if (crc_out) lane0_store_u32(crc_out + b, crc);
      if (flags & kFlagStamp)
        lane0_store_u32(const_cast<uint32_t *>(reinterpret_cast<const uint32_t *>(base + b * stride)), crc);
      if (first_bad && uni(sw) != crc) {
        if (bad_bitmap) lane0_atomic_or(bad_bitmap + (b >> 5), 1u << (b & 31));
        if (b < reported) lane0_atomic_umin64(first_bad, b);
        reported = b < reported ? b : reported;
      }
    }
    if (!nv) return;
    // next piece: p1 <- p2, p2 <- hand-out
    pc = p1;
    kc = k1;
    gp = npa;
    p1 = p2;
    k1 = k2;
    k2 = uni(k3v);
    if (lane == 0) k3v = atomicAdd(&s_next, 1u);
    p2 = pc_of(k2);
  }
}

// ---------------------------------------------------------------------------
// k_frame_np (A/B, tools/kframe): AddCRCsToData framing by short-lived 4-wave
// workgroups, as the non-persistent copies that reach 5.6-6.0 TB/s do
// (DESIGN 4.4a), instead of one persistent 16-wave workgroup per CU.  That
// needs tables small enough for several workgroups per CU: the row-shift
// tables with kR replicas (lane l reads replica l % kR; bank (v*kR + l % kR) %
// 32, so 32/kR lanes of a half-wave spread over 32/kR banks), the 4-byte shift
// tables unreplicated and the lane-placement columns, 16 + 4 + 8 KiB at kR = 4.
// Wave w of workgroup g frames interior blocks (g*4 + w)*kPer + k + 1: its rows
// are loaded first, in flight while the workgroup fills its tables.
template <int kR = 4, int kPer = 1>
__global__ __launch_bounds__(256) void k_frame_np(const uint8_t *__restrict__ src, uint64_t n,
                                                  uint8_t *__restrict__ dst, uint64_t nblk,
                                                  uint32_t *__restrict__ crc_out,
                                                  const DeviceTables *__restrict__ tables) {
  static_assert(kR == 1 || kR == 2 || kR == 4 || kR == 8, "replicas");
  __shared__ __attribute__((aligned(16))) uint32_t tm[4 * 256 * kR];  // [t][v][replica]
  __shared__ __attribute__((aligned(16))) uint32_t ts4[4 * 256];      // [t][v]
  __shared__ uint32_t tl[32 * 64];                                     // [i][lane]
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  constexpr uint64_t kPay = 4092;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = uni(tid >> 6);
  const uint64_t ni = nblk > 2 ? nblk - 2 : 0;
  const uint64_t i0 = ((uint64_t)blockIdx.x * 4 + wave) * kPer;
  // 1) this wave's rows (past the end: re-read interior block 0, never stored)
  u32x4 v[kPer][4];
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint64_t i = i0 + k < ni ? i0 + k : 0;
    const uint8_t *S = src + (i + 1) * kPay - 4 + 16u * lane;
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (ni) v[k][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(S + r * kRowBytes));
  }
  // 2) tables into LDS while the rows are in flight
  {
    const uint32_t *tg = &tables->tg[0][0];
    for (uint32_t e = tid; e < 1024; e += 256) {
      const uint32_t x = tg[e];
#pragma unroll
      for (int q = 0; q < kR; q++) tm[e * kR + q] = x;
    }
    const uint32_t *s4 = &tables->s4[0][0];
    for (uint32_t e = tid; e < 1024; e += 256) ts4[e] = s4[e];
    const uint32_t *lt = &tables->lane[0][0];
    for (uint32_t e = tid; e < 2048; e += 256) tl[(e & 31u) * 64 + (e >> 5)] = lt[e];
  }
  const uint32_t w0 = tables->w0;
  __syncthreads();
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tl[i * 64 + lane];
  const uint32_t rep4 = (lane % kR) * 4u;
  // shift(c, 1024) = tg[0][c0] ^ tg[1][c1] ^ tg[2][c2] ^ tg[3][c3]: byte address
  // t*1024*kR + v*4*kR + 4*(l % kR)
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    constexpr uint32_t E = 4u * kR, T = 1024u * kR;
    const uint32_t t0 = lds_u32(tm, ((c & 255u) * E) | rep4);
    const uint32_t t1 = lds_u32(tm, T + ((((c >> 8) & 255u) * E) | rep4));
    const uint32_t t2 = lds_u32(tm, 2 * T + ((((c >> 16) & 255u) * E) | rep4));
    const uint32_t t3 = lds_u32(tm, 3 * T + (((c >> 24) * E) | rep4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    return xor3(xor3(ts4[x & 255u], ts4[256 + ((x >> 8) & 255u)], ts4[512 + ((x >> 16) & 255u)]),
                ts4[768 + (x >> 24)], w);
  };
  // 3) store, hash, finalize
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    if (i0 + k >= ni) break;  // wave-uniform
    const uint64_t b = i0 + k + 1;
    uint8_t *ob = dst + b * (uint64_t)HC_FRAME_BLOCK + 16u * lane;
    uint32_t cc[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 x = v[k][r];
      if (r == 0) x.x = lane == 0 ? 0u : x.x;  // bytes 0..3: zeros now, the CRC below
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(ob + r * kRowBytes));
      if (r == 0) x.x = lane == 0 ? w0 : x.x;  // Go's init in place of the CRC field
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int q = 0; q < 4; q++) cc[q] = r == 0 ? w[q] : row_step(cc[q], w[q]);
    }
    const uint32_t dd = shift4(shift4(shift4(cc[0], cc[1]), cc[2]), cc[3]);
    const uint32_t crcv = wave_xor(matvec32(col, dd)) ^ 0xFFFFFFFFu;
    lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crcv);
    if (crc_out) lane0_store_u32(crc_out + b, crcv);
  }
  // 4) the edge blocks: workgroup 0's waves 0 and 1
  if (blockIdx.x == 0 && wave < 2 && (wave == 0 || nblk > 1)) {
    const uint64_t b = wave == 0 ? 0 : nblk - 1;
    uint32_t c[4];
    uint4 keep;
    frame_edge_rows(b, src, n, dst, lane, w0, row_step, c, keep);
    const uint32_t dd = shift4(shift4(shift4(c[0], c[1]), c[2]), c[3]);
    const uint32_t crcv = wave_xor(matvec32(col, dd)) ^ 0xFFFFFFFFu;
    if (lane == 0) {
      keep.x = crcv;
      *reinterpret_cast<uint4 *>(dst + b * (uint64_t)HC_FRAME_BLOCK) = keep;
      if (crc_out) crc_out[b] = crcv;
    }
  }
}

}  // namespace
}  // namespace hc
