# k_unframe 16 KiB: 8-wave workgroups taking two blocks 4 apart (the 8 KiB
# form's layout: workgroup L takes blocks 8 (L / 4) + L % 4 and that + 4),
# instead of one block per 4-wave workgroup
SUBS = [("__global__ __launch_bounds__(256) void k_unframe(",
         "__global__ __launch_bounds__(lg_groups == 2 ? 512 : 256) void k_unframe("),
        ("  for (uint32_t k = 0; k < kPer; k++) t[k] = g[threadIdx.x + k * 256u];",
         "  for (uint32_t k = 0; k < kPer; k++) t[k] = g[(threadIdx.x & 255u) + k * 256u];"),
        ("  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[threadIdx.x + k * 256u] = t[k];",
         "  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[(threadIdx.x & 255u) + k * 256u] = t[k];"),
        ("    __shared__ uint32_t reg[4], st_word[4];", "    __shared__ uint32_t reg[8], st_word[4];"),
        ("                                      : ((uint64_t)L * 4 + wave) >> lg_groups;",
         "                                      : 8ull * (L >> 2) + (L & 3u) + 4u * (wave >> 2);"),
        ("  const uint64_t grid = unframe_grid(nblk, lg_groups);  // one 4 KiB group per wave, 4 waves per workgroup",
         "  const uint64_t grid = lg_groups == 2 ? 4 * ((nblk + 7) / 8) : unframe_grid(nblk, lg_groups);"),
        ("  hipLaunchKernelGGL((k_unframe<L>), dim3((unsigned)grid), dim3(256), 0, s,",
         "  hipLaunchKernelGGL((k_unframe<L>), dim3((unsigned)grid), dim3(L == 2 ? 512 : 256), 0, s,")]
