# k_frame in 8-wave workgroups: one load of the placement columns into LDS per
# 8 interior blocks instead of 4; a workgroup's eight waves take blocks
# kFrameSpread apart (one source alignment, as before)
SUBS = [("__global__ __launch_bounds__(256) void k_frame(",
         "__global__ __launch_bounds__(512) void k_frame("),
        ("  for (uint32_t k = 0; k < kPer; k++) t[k] = g[threadIdx.x + k * 256u];",
         "  for (uint32_t k = 0; k < kPer; k++) t[k] = g[(threadIdx.x & 255u) + k * 256u];"),
        ("  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[threadIdx.x + k * 256u] = t[k];",
         "  for (uint32_t k = 0; k < kPer; k++) reinterpret_cast<uint4 *>(lq)[(threadIdx.x & 255u) + k * 256u] = t[k];"),
        ("  const uint64_t b = 1 + 4ull * kFrameSpread * (I / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + I % kFrameSpread;",
         "  const uint64_t b = 1 + 8ull * kFrameSpread * (I / kFrameSpread) + kFrameSpread * uni(threadIdx.x >> 6) + I % kFrameSpread;"),
        ("  const uint4 lq0 = lqg[threadIdx.x], lq1 = lqg[threadIdx.x + 256u];",
         "  const uint4 lq0 = lqg[threadIdx.x & 255u], lq1 = lqg[(threadIdx.x & 255u) + 256u];"),
        ("  reinterpret_cast<uint4 *>(lq)[threadIdx.x] = lq0;\n  reinterpret_cast<uint4 *>(lq)[threadIdx.x + 256u] = lq1;",
         "  reinterpret_cast<uint4 *>(lq)[threadIdx.x & 255u] = lq0;\n  reinterpret_cast<uint4 *>(lq)[(threadIdx.x & 255u) + 256u] = lq1;"),
        ("  const uint64_t wgs = 1 + (nblk > 2 ? kFrameSpread * ((nblk - 2 + 4 * kFrameSpread - 1) / (4 * kFrameSpread)) : 0);",
         "  const uint64_t wgs = 1 + (nblk > 2 ? kFrameSpread * ((nblk - 2 + 8 * kFrameSpread - 1) / (8 * kFrameSpread)) : 0);"),
        ("  hipLaunchKernelGGL(k_frame, dim3((unsigned)wgs), dim3(256), 0, s,",
         "  hipLaunchKernelGGL(k_frame, dim3((unsigned)wgs), dim3(512), 0, s,")]
