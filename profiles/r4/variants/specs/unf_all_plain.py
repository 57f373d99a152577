# k_unframe 4 KiB: every payload store plain (not non-temporal)
SUBS = [("    for (int r = 0; r < 4; r++) __builtin_nontemporal_store(sv[r], reinterpret_cast<u32x4_u *>(sa[r]));\n",
         "    for (int r = 0; r < 4; r++) *reinterpret_cast<u32x4_u *>(sa[r]) = sv[r];\n")]
