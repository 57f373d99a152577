# k_unframe 8/16 KiB: group 0's lane-0 row-0 bytes 4..15 by a 12-B buffer store,
# the row-0 16-B store through a buffer range in which that lane is out of
# range (no overlapping store)
SUBS = [("""        const uint32_t nx = __builtin_amdgcn_update_dpp(0u, t.x, 0x101, 0xF, 0xF, false);  // lane+1's x
        if (head) st_word[wave >> lg_groups] = t.x;                                           // LE32(block[0:4])
        const u32x4 first = {t.y, t.z, t.w, nx};
        sv[r] = head ? first : t;
        t.x = head ? w0 : t.x;  // Go's init in place of the CRC field
""", """        if (head) st_word[wave >> lg_groups] = t.x;  // LE32(block[0:4])
        t.x = head ? w0 : t.x;                       // Go's init in place of the CRC field
"""),
        ("""#pragma unroll
    for (int r = 0; r < 4; r++)
      __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(ob + r * kRowBytes + (r == 0 && head ? 4 : 0)));
""", """    {
      typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
      const __amdgpu_buffer_rsrc_t r0 = buf_range(ob - 16u * lane, kRowBytes);
      __builtin_amdgcn_raw_buffer_store_b128(sv[0], r0, head ? 2u * kRowBytes : 16u * lane, 0, 2);
      const __amdgpu_buffer_rsrc_t rh = buf_range(out + b * Bp, 12u);
      __builtin_amdgcn_raw_buffer_store_b96(u32x3{sv[0].y, sv[0].z, sv[0].w}, rh, head ? 0u : 16u, 0, 2);
    }
#pragma unroll
    for (int r = 1; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(ob + r * kRowBytes));
""")]
