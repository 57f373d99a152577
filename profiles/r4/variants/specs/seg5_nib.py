# k_seg_stream's 4-byte shifts through nibble tables with 32 replicas
# (conflict-free: 8 lookups a shift instead of 4 byte lookups on 4 replicas),
# written over the byte tables' 16 KiB after the shared fill
NIB = [
("""  fill_crc_tables(lds, tables, tid, kFastThreads);
  if (tid """, """  {  // the row tables as fill_crc_tables; nibble tables [p][v][r] where it puts the byte tables
    const uint32_t *tg = &tables->tg[0][0];
    for (uint32_t q = tid; q < kLdsMainBytes / 16; q += kFastThreads) {
      const uint32_t a = q * 16;
      const uint32_t k = ((a >> 16) << 1) | ((a >> 7) & 1u);
      const uint32_t v = tg[k * 256 + ((a >> 8) & 255u)];
      *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + a) = make_uint4(v, v, v, v);
    }
    const uint32_t p = tid >> 7, v = (tid >> 3) & 15u;
    const uint32_t e = tables->s4[p >> 1][v << (4 * (p & 1u))];
    *reinterpret_cast<uint4 *>(lds + kLdsMainBytes / 4 + (p * 16 + v) * 32 + (tid & 7u) * 4) = make_uint4(e, e, e, e);
  }
  if (tid """),
("""  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, S4base + ((x & 255u) << 4));
    const uint32_t t1 = lds_u32(lds, S4base + 4096u + (((x >> 8) & 255u) << 4));
    const uint32_t t2 = lds_u32(lds, S4base + 8192u + (((x >> 16) & 255u) << 4));
    const uint32_t t3 = lds_u32(lds, S4base + 12288u + ((x >> 24) << 4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  // lane chunk (4 words) -> its raw CRC""", """  const uint32_t NBbase = kLdsMainBytes + ((lane & 31u) << 2);
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    uint32_t t[8];
#pragma unroll
    for (int p = 0; p < 8; p++) t[p] = lds_u32(lds, NBbase + 2048u * p + (((x >> (4 * p)) & 15u) << 7));
    return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), xor3(t[6], t[7], w));
  };
  // lane chunk (4 words) -> its raw CRC"""),
]
SUBS = NIB
