# k_unframe at every size in 8-wave workgroups (one LDS fill of the placement
# columns per 8 waves instead of 4): 4 KiB eight blocks kFrameSpread apart
# (one output alignment), 8 KiB four blocks 4 apart, 16 KiB two blocks 4 apart
SUBS = [("__global__ __launch_bounds__(256) void k_unframe(",
         "__global__ __launch_bounds__(512) void k_unframe("),
        ("  for (uint32_t k = 0; k < kPer; k++) t[k] = g[threadIdx.x + k * 256u];",
         "  for (uint32_t k = 0; k < kPer; k++) t[k] = g[(threadIdx.x & 255u) + k * 256u];"),
        ("  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[threadIdx.x + k * 256u] = t[k];",
         "  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[(threadIdx.x & 255u) + k * 256u] = t[k];"),
        ("    const uint64_t b = 4ull * kFrameSpread * (L / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + L % kFrameSpread;",
         "    const uint64_t b = 8ull * kFrameSpread * (L / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + L % kFrameSpread;"),
        ("    __shared__ uint32_t reg[4], st_word[4];", "    __shared__ uint32_t reg[8], st_word[4];"),
        ("    const uint64_t b = lg_groups == 1 ? 8ull * (L >> 2) + (L & 3u) + 4u * (wave >> 1)\n"
         "                                      : ((uint64_t)L * 4 + wave) >> lg_groups;",
         "    const uint64_t b = lg_groups == 1 ? 16ull * (L >> 2) + (L & 3u) + 4u * (wave >> 1)\n"
         "                                      : 8ull * (L >> 2) + (L & 3u) + 4u * (wave >> 2);"),
        ("  const uint64_t grid = unframe_grid(nblk, lg_groups);  // one 4 KiB group per wave, 4 waves per workgroup",
         "  const uint64_t grid = lg_groups == 0 ? kFrameSpread * ((nblk + 8 * kFrameSpread - 1) / (8 * kFrameSpread))\n"
         "                       : lg_groups == 1 ? 4 * ((nblk + 15) / 16) : 4 * ((nblk + 7) / 8);"),
        ("  hipLaunchKernelGGL((k_unframe<L>), dim3((unsigned)grid), dim3(256), 0, s,",
         "  hipLaunchKernelGGL((k_unframe<L>), dim3((unsigned)grid), dim3(512), 0, s,")]
