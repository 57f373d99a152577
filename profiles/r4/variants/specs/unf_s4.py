# k_unframe 4 KiB: workgroup L takes blocks 4 (4 (L / 4) + w) + L % 4 (production: 8);
# with the L2's partial-write counts, which boundaries leave the L2 partially written
SUBS = [("    const uint64_t b = 4ull * kFrameSpread * (L / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + L % kFrameSpread;\n",
         "    const uint64_t b = 4ull * 4u * (L / 4u) + 4u * uni(threadIdx.x >> 6) + L % 4u;\n")]
