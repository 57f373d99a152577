# k_unframe 4 KiB: workgroup L takes blocks 2 (4 (L / 2) + w) + L % 2 (production: 8);
# with the L2's partial-write counts, which boundaries leave the L2 partially written
SUBS = [("    const uint64_t b = 4ull * kFrameSpread * (L / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + L % kFrameSpread;\n",
         "    const uint64_t b = 4ull * 2u * (L / 2u) + 2u * uni(threadIdx.x >> 6) + L % 2u;\n")]
