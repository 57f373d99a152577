// Does a 16-byte LDS read at a byte address that is not 16-B (or 4-B) aligned
// return the bytes at that address on gfx950?  (k_md5 could then read a
// message's words at its byte phase inside an aligned stage image.)
//   hipcc --offload-arch=gfx950 -O2 tools/lds_unaligned_probe.hip -o tools/build/lds_unaligned_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void probe(uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t s[2048];
  for (uint32_t i = threadIdx.x; i < 2048; i += blockDim.x) s[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  const uint32_t off = threadIdx.x * 17u;  // every byte phase mod 16 across the lanes
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = *reinterpret_cast<const u32x4 *>(s + off);
  const uint32_t w = *reinterpret_cast<const uint32_t *>(s + off + 1);
  out[threadIdx.x * 5 + 0] = v.x;
  out[threadIdx.x * 5 + 1] = v.y;
  out[threadIdx.x * 5 + 2] = v.z;
  out[threadIdx.x * 5 + 3] = v.w;
  out[threadIdx.x * 5 + 4] = w;
}

int main() {
  uint32_t *d = nullptr;
  if (hipMalloc(&d, 64 * 5 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[64 * 5];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  int bad = 0;
  for (uint32_t l = 0; l < 64; l++) {
    const uint32_t off = l * 17u;
    auto byte = [](uint32_t i) { return (uint32_t)(uint8_t)(i * 7 + 3); };
    for (int k = 0; k < 4; k++) {
      const uint32_t want = byte(off + 4 * k) | byte(off + 4 * k + 1) << 8 | byte(off + 4 * k + 2) << 16 |
                            byte(off + 4 * k + 3) << 24;
      if (h[l * 5 + k] != want) bad++;
    }
    const uint32_t want1 = byte(off + 1) | byte(off + 2) << 8 | byte(off + 3) << 16 | byte(off + 4) << 24;
    if (h[l * 5 + 4] != want1) bad++;
  }
  printf("{\"probe\": \"lds_unaligned\", \"mismatches\": %d, \"of\": %d}\n", bad, 64 * 5);
  hipFree(d);
  return 0;
}
