# k_frame: every row stored after the hash (rows 1-3 first, then row 0 with
# the CRC); production stores rows 1-3 before the hash
SUBS = [("#pragma unroll\n  for (int r = 1; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4 *>(ob + r * kRowBytes));\n  uint32_t c[4];\n",
         "  uint32_t c[4];\n"),
        ("  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;\n  u32x4 t0 = v[0];\n",
         "  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;\n#pragma unroll\n  for (int r = 1; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4 *>(ob + r * kRowBytes));\n  u32x4 t0 = v[0];\n")]
