SUBS = [("""  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    return matvec32(col, shift4(shift4(shift4(a, b_), c), d));
  };""", """  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    const uint32_t v = shift4(shift4(shift4(a, b_), c), d);
    uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0;
#pragma unroll
    for (int i = 0; i < 32; i += 4) {
      e0 = __builtin_amdgcn_bitop3_b32((uint32_t)((int32_t)(v << (31 - i)) >> 31), col[i], e0, 0x6A);
      e1 = __builtin_amdgcn_bitop3_b32((uint32_t)((int32_t)(v << (30 - i)) >> 31), col[i + 1], e1, 0x6A);
      e2 = __builtin_amdgcn_bitop3_b32((uint32_t)((int32_t)(v << (29 - i)) >> 31), col[i + 2], e2, 0x6A);
      e3 = __builtin_amdgcn_bitop3_b32((uint32_t)((int32_t)(v << (28 - i)) >> 31), col[i + 3], e3, 0x6A);
    }
    return xor3(e0, e1, e2) ^ e3;
  };""")]
