// VALU issue rate of MD5's integer instruction mix against f32 FMA on gfx950
// (is k_md5's 0.204 wave-instructions per SIMD-cycle near the
// integer ceiling?).  8 independent chains per lane, 8 waves per SIMD
// (2048 threads per CU), timed with HIP events; prints wave-instructions per
// second for each mix and the ratio.  Outputs are stored so nothing folds.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o tools/valu_rate tools/valu_rate.hip
// (-fno-slp-vectorize: the f32 chains stay one v_fma each, not v_pk_fma_f32)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kIters = 1 << 14;
constexpr int kChains = 8;

__global__ __launch_bounds__(512) void k_int(uint32_t *out, uint32_t seed) {
  uint32_t a[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) a[i] = seed + threadIdx.x * 7u + i;
  const uint32_t b = seed ^ 0x5bd1e995u, c = seed * 3u;
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int i = 0; i < kChains; i++) {  // 4 ops per chain: bitop3, add3, alignbit, add (an MD5 step)
      uint32_t f = __builtin_amdgcn_bitop3_b32(a[i], b, c, 0xCA);
      f = f + a[i] + 0x9e3779b9u;
      f = __builtin_amdgcn_alignbit(f, f, 25);
      a[i] = f + b;
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(512) void k_f32(float *out, float seed) {
  float a[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) a[i] = seed + threadIdx.x * 0.5f + i;
  const float b = seed * 0.999f, c = 1e-7f;
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int i = 0; i < kChains; i++) {  // 4 dependent FMAs per chain
      a[i] = __builtin_fmaf(a[i], b, c);
      a[i] = __builtin_fmaf(a[i], b, c);
      a[i] = __builtin_fmaf(a[i], b, c);
      a[i] = __builtin_fmaf(a[i], b, c);
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int wgs = cus * 4;  // 4 x 512 threads = 2048 per CU = 8 waves per SIMD
  void *buf;
  hipMalloc(&buf, (size_t)wgs * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double waves = (double)wgs * 512 / 64;
  const double insts = waves * kIters * kChains * 4;  // wave-instructions in the loops
  double rate[2];
  for (int k = 0; k < 2; k++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      if (k == 0)
        hipLaunchKernelGGL(k_int, dim3(wgs), dim3(512), 0, 0, (uint32_t *)buf, 1234u + rep);
      else
        hipLaunchKernelGGL(k_f32, dim3(wgs), dim3(512), 0, 0, (float *)buf, 1.5f + rep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      rate[k] = insts / (ms * 1e-3);
    }
    const double per_simd_ghz = rate[k] / (cus * 4.0) / 1e9;
    printf("{\"mix\": \"%s\", \"wave_insts_per_s\": %.4g, \"per_simd_per_ns\": %.4f}\n", k == 0 ? "int_md5_step" : "f32_fma",
           rate[k], per_simd_ghz);
  }
  printf("{\"int_over_f32\": %.3f, \"cus\": %d}\n", rate[0] / rate[1], cus);
  hipFree(buf);
  return 0;
}
