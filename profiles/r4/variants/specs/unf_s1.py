# k_unframe 4 KiB: workgroup L takes blocks 1 (4 (L / 1) + w) + L % 1 (production: 8);
# with the L2's partial-write counts, which boundaries leave the L2 partially written
SUBS = [("    const uint64_t b = 4ull * kFrameSpread * (L / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + L % kFrameSpread;\n",
         "    const uint64_t b = 4ull * 1u * (L / 1u) + 1u * uni(threadIdx.x >> 6) + L % 1u;\n")]
