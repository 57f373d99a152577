# k_crc_grp / k_crc_fast rows with plain (cached) loads instead of nontemporal
SUBS = [("  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(row + lane * 16u));",
         "  const u32x4 v = *reinterpret_cast<const u32x4 *>(row + lane * 16u);")]
