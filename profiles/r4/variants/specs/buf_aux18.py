# buffer row loads (k_seg_stream, k_crc_any) with cache policy 18 instead of 2 (nt)
SUBS = [("  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 2));",
         "  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 18));")]
