LDSCOL = [
("""  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4 + kFastWaves * 64];
  __shared__ uint32_t s_next;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  fill_crc_tables(lds, tables, tid, kFastThreads);
  if (tid == 0) s_next = 2 * kFastWaves;  // indices 0 .. 2W-1 are dealt statically below
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
""", """  constexpr uint32_t kColBase = kFastLdsBytes / 4 + kFastWaves * 64;  // colT[i][lane]
  __shared__ __attribute__((aligned(16))) uint32_t lds[kColBase + 32 * 64];
  __shared__ uint32_t s_next;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  fill_crc_tables(lds, tables, tid, kFastThreads);
  if (tid == 0) s_next = 2 * kFastWaves;  // indices 0 .. 2W-1 are dealt statically below
  {
    const uint32_t t0 = tables->lane[tid & 63][tid >> 6], t1 = tables->lane[tid & 63][16 + (tid >> 6)];
    lds[kColBase + tid] = t0;
    lds[kColBase + 1024 + tid] = t1;
  }
"""),
("""  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    return matvec32(col, shift4(shift4(shift4(a, b_), c), d));
  };""", """  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    const uint32_t v = shift4(shift4(shift4(a, b_), c), d);
    const uint32_t *ct = lds + kColBase + lane;
    uint32_t e = 0;
#pragma unroll
    for (int i = 0; i < 32; i++)
      e = __builtin_amdgcn_bitop3_b32((uint32_t)((int32_t)(v << (31 - i)) >> 31), ct[i * 64], e, 0x6A);
    return e;
  };"""),
]
SUBS = LDSCOL
