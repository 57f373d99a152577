# k_unframe 4 KiB: rows 0 and 3 (the lines shared with the neighbouring blocks'
# outputs) with plain stores, rows 1-2 non-temporal (r4jj: 1.27M partial
# 32-B write requests per 1M blocks, against 0.53M at 8 KiB)
SUBS = [("    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));\n",
         "    for (int r = 0; r < 4; r++) {\n"
         "      if (r == 0 || r == 3) *reinterpret_cast<u32x4_u *>(sa[r]) = sv[r];\n"
         "      else __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));\n"
         "    }\n")]
