# k_unframe 4 KiB: no overlapping head store.  Lane l's 16 output bytes of row r
# are payload bytes 4 + 16 l .. 19 + 16 l of the row (its own x..w minus x, plus
# lane l+1's x by DPP wave_shl:1; lane 63 takes the next row's lane 0 x), at
# out + b (B-4) + 1024 r + 16 l.  The block's last 12 bytes (row 3, lane 63)
# go out by a 12-B buffer store; row 3's 16-B store runs through a buffer range
# that ends at the block's last payload byte, which drops lane 63's.
# (r4jj/r4nn: 1.27M partial write requests per 1M blocks whatever the spread;
# 0.53M per 0.5M 8 KiB blocks: one per head store.)
SUBS = [("""    uint8_t *ob = out + b * Bp + 16u * lane - 4;
    u32x4 sv[4];
    uint8_t *sa[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      if (r == 0) {
        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);  // lane+1's x
        stored = __builtin_amdgcn_readfirstlane(t.x);                                         // LE32(block[0:4])
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = lane == 0 ? first : t;
        sa[r] = ob + (lane == 0 ? 4 : 0);
        t.x = lane == 0 ? w0 : t.x;  // Go's init in place of the CRC field
      } else {
        sv[r] = t;
        sa[r] = ob + r * kRowBytes;
      }
""", """    uint8_t *ob = out + b * Bp + 16u * lane;
    u32x4 sv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      u32x4 t = v[r];
      uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x130, 0xF, 0xF, false);  // lane+1's x (wave_shl:1)
      const uint32_t nr = r < 3 ? __builtin_amdgcn_readlane(v[r < 3 ? r + 1 : 3].x, 0) : 0u;
      nx = lane == 63 ? nr : nx;
      sv[r] = u32x4{t.y, t.z, t.w, nx};
      if (r == 0) {
        stored = __builtin_amdgcn_readfirstlane(t.x);  // LE32(block[0:4])
        t.x = lane == 0 ? w0 : t.x;                    // Go's init in place of the CRC field
      }
"""),
        ("""    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
""", """    for (int r = 0; r < 3; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(ob + r * kRowBytes));
    {
      const __amdgpu_buffer_rsrc_t rb = buf_range(out + b * Bp, (uint32_t)Bp);
      __builtin_amdgcn_raw_buffer_store_b128(sv[3], rb, 3u * kRowBytes + 16u * lane, 0, 2);
      typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
      __builtin_amdgcn_raw_buffer_store_b96(u32x3{sv[3].x, sv[3].y, sv[3].z}, rb, lane == 63 ? 4080u : (uint32_t)Bp, 0, 2);
    }
""")]
