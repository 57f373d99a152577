# k_md5 with 3-block stages, one stage in flight and three workgroups per CU
# (12 waves: 3 per SIMD; LDS 3 x 52 KiB, VGPRs <= 168)
SUBS = [
    ("constexpr int kMd5StageBlocks = 4;  // 64-byte blocks per lane per stage",
     "constexpr int kMd5StageBlocks = 3;  // 64-byte blocks per lane per stage"),
    ("template <bool kOff, bool kLen, int kStage = kMd5StageBlocks, int kDepth = 2, bool kTable = true>",
     "template <bool kOff, bool kLen, int kStage = kMd5StageBlocks, int kDepth = 1, bool kTable = true>"),
    ("  if (grid > (uint64_t)cus * 2) grid = (uint64_t)cus * 2;",
     "  if (grid > (uint64_t)cus * 3) grid = (uint64_t)cus * 3;"),
]
