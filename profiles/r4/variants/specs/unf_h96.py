# k_unframe 4 KiB: lane 0's row-0 bytes 4..15 by a 12-B buffer store, the
# row-0 16-B store through a buffer range in which lane 0 is out of range (no
# overlapping store; the other lanes' layout unchanged)
SUBS = [("""        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);  // lane+1's x
        stored = __builtin_amdgcn_readfirstlane(t.x);                                         // LE32(block[0:4])
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = lane == 0 ? first : t;
        sa[r] = ob + (lane == 0 ? 4 : 0);
""", """        stored = __builtin_amdgcn_readfirstlane(t.x);  // LE32(block[0:4])
        sv[r] = t;
        sa[r] = ob;
"""),
        ("""#pragma unroll
    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
""", """    {
      typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
      const __amdgpu_buffer_rsrc_t r0 = buf_range(out + b * Bp - 4, kRowBytes);
      __builtin_amdgcn_raw_buffer_store_b128(sv[0], r0, lane == 0 ? 2u * kRowBytes : 16u * lane, 0, 2);
      const __amdgpu_buffer_rsrc_t rh = buf_range(out + b * Bp, 12u);
      __builtin_amdgcn_raw_buffer_store_b96(u32x3{sv[0].y, sv[0].z, sv[0].w}, rh, lane == 0 ? 0u : 16u, 0, 2);
    }
#pragma unroll
    for (int r = 1; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));
""")]
