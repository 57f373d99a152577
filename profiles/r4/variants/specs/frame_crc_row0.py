# k_frame: row 0 stored after the hash with the CRC in lane 0's word (one full
# store of the block's first line instead of a zero word now and a 4-byte CRC
# store later: r4jj, 0.77M partial 32-B write requests per 1M blocks)
SUBS = [("  for (int r = 0; r < 4; r++) {  // lane 0 writes zeros to bytes 0..3 and the CRC over them below\n"
         "    u32x4 t = v[r];\n"
         "    if (r == 0) t.x = lane == 0 ? 0u : t.x;\n"
         "    __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob + r * kRowBytes));\n"
         "  }\n",
         "  for (int r = 1; r < 4; r++) __builtin_nontemporal_store(v[r], reinterpret_cast<u32x4 *>(ob + r * kRowBytes));\n"),
        ("  lane0_store_u32(reinterpret_cast<uint32_t *>(ob), crcv);  // lane 0's ob is the block start\n",
         "  {\n"
         "    u32x4 t = v[0];\n"
         "    t.x = lane == 0 ? crcv : t.x;\n"
         "    __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(ob));\n"
         "  }\n")]
