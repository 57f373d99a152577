// kgrp4.hip -- what k_crc_grp's per-block finalise costs (late round 3).
// At 4 KiB the streaming kernel trails 8 KiB by ~2.4 points; the finalise (three
// 4-byte shifts through LDS, the lane placement's 32x32 mat-vec in VGPRs, a
// wave XOR) runs once per block.  tools/gen_grp_fin.py copies the product
// kernel with a switch on the finalise: the copy (words checked), timing-only
// builds without the placement and without the whole finalise.
//
//   ./kgrp4 [nblocks=1000000] [block=4096] [rounds=6] [launches=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <numeric>
#include <string>
#include <vector>

#include "../hunddb_amd/csrc/hc_kernels.hip"
#include "build/k_crc_grp_fin.inc"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

namespace {
struct Variant {
  std::string name;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const uint32_t B = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 4096;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 6;
  const int launches = argc > 4 ? std::atoi(argv[4]) : 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("device %s, %d CUs; %llu x %u B = %.1f GB\n", prop.gcnArchName, cus, (unsigned long long)N, B,
              N * (double)B / 1e9);
  uint8_t *buf;
  uint32_t *crc;
  hc::DeviceTables *dt;
  CK(hipMalloc(&buf, N * (uint64_t)B));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hc::launch_fill(buf, nullptr, nullptr, B, B, N, 0x48756E64, cus * 16, s));
  CK(hipStreamSynchronize(s));
  hc::Batch b{};
  b.base = buf;
  b.stride = B;
  b.ulen = B;
  b.nblocks = N;
  b.crc_out = crc;
  b.tables = dt;
  std::vector<Variant> vs;
  const uint32_t lg = hc::grp_lg_chunk(N, cus, B);  // production's chunk
  const bool xcd = hc::grp_xcd(B, cus, N);          // production's slot order
  auto fin = [&](int f) {
    return [&, f](hipStream_t st) {
#define FIN(X, F)                                                                                                  \
  hipLaunchKernelGGL((hc::k_crc_grp_fin<false, X, F>), dim3(cus), dim3(hc::kFastThreads), 0, st, b.base, nullptr,  \
                     nullptr, b.stride, b.ulen, 0u, N, lg, crc, nullptr, nullptr, dt, nullptr)
      if (xcd) {
        if (f == 0) FIN(true, 0); else if (f == 1) FIN(true, 1); else FIN(true, 2);
      } else {
        if (f == 0) FIN(false, 0); else if (f == 1) FIN(false, 1); else FIN(false, 2);
      }
#undef FIN
    };
  };
  for (int k = 0; k < 2; k++) {
    vs.push_back({"PROD launch_grp", [&](hipStream_t st) { CK(hc::launch_grp(b, cus, st)); }, {}});
    vs.push_back({"copy (kFin 0)", fin(0), {}});
    vs.push_back({"NULL placement (shift4 kept)", fin(2), {}});
    vs.push_back({"NULL finalise", fin(1), {}});
  }
  std::vector<uint32_t> ref(N), got(N);
  vs[0].run(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), crc, N * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto &v : vs) {
    if (v.name.rfind("NULL", 0) == 0) continue;  // timing-only builds
    CK(hipMemsetAsync(crc, 0, N * 4, s));
    v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), crc, N * 4, hipMemcpyDeviceToHost));
    if (got != ref) {
      std::printf("MISMATCH in variant %s\n", v.name.c_str());
      bad++;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs)
      for (int l = 0; l < launches; l++) {
        CK(hipEventRecord(e0, s));
        v.run(s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms);
      }
  std::printf("%-40s %10s %10s %8s %9s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double bytes = (double)N * B;
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-40s %10.1f %10.1f %7.2f%% %9.4f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6,
                bytes / med / 1e6 / 80.0, med);
  }
  return bad ? 3 : 0;
}
