# k_frame: rows 1-3 stored after the row folds, before the stream combine and
# the lane placement (production: before the folds)
SUBS = [("#pragma unroll\n  for (int r = 1; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4 *>(ob + r * kRowBytes));\n  uint32_t c[4];\n",
         "  uint32_t c[4];\n"),
        ("  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);\n  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;\n  u32x4 t0 = v[0];\n",
         "#pragma unroll\n  for (int r = 1; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4 *>(ob + r * kRowBytes));\n  const uint32_t d = xapply(TS, xapply(TS, xapply(TS, c[0], c[1]), c[2]), c[3]);\n  const uint32_t crcv = wave_xor(place_lq(lq, lane, d)) ^ 0xFFFFFFFFu;\n  u32x4 t0 = v[0];\n")]
