// kgrp3.hip -- round-3 study of k_crc_grp's large-batch drop (configs[3] at
// N = 1: 16M x 8 KiB runs ~0.7-2 % below 1M x 8 KiB).  PMC passes over the
// production kernel (profiles/r3/pmc_size/) ruled out address translation
// (UTCL1 misses per GB fall with size) and showed the L2's DRAM-credit stalls
// per read request doubling at 16M.  At any moment the G workgroups stream G
// neighbouring chunks (one 256 MiB window of the buffer); this harness tests
// whether spreading the concurrently streamed chunks over the whole buffer
// changes that: chunk slot q -> (q * perm) mod nchunks (tools/gen_grp_perm.py
// copies the product kernel and permutes only that).
//
//   ./kgrp3 [nblocks=16000000] [block=8192] [rounds=4] [launches=3]
//
// Every variant's CRC words are compared with production's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <numeric>
#include <string>
#include <vector>

#include "../hunddb_amd/csrc/hc_kernels.hip"
#include "build/k_crc_grp_perm.inc"

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
uint64_t coprime_near(uint64_t target, uint64_t q) {
  if (target < 1) target = 1;
  for (uint64_t p = target;; p++)
    if (std::gcd(p, q) == 1) return p;
}
}  // namespace

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 16000000;
  const uint32_t B = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 8192;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 4;
  const int launches = argc > 4 ? std::atoi(argv[4]) : 3;
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
  vs.push_back({"PROD launch_grp", [&](hipStream_t st) { CK(hc::launch_grp(b, cus, st)); }, {}});
  auto perm = [&](uint32_t lg, uint64_t p, bool xcd) {
    const uint64_t q = N >> lg;
    return [&, lg, p, q, xcd](hipStream_t st) {
      if (xcd)
        hipLaunchKernelGGL((hc::k_crc_grp_perm<false, true>), dim3(cus), dim3(hc::kFastThreads), 0, st, b.base, nullptr,
                           nullptr, b.stride, b.ulen, 0u, N, lg, crc, nullptr, nullptr, dt, p, q);
      else
        hipLaunchKernelGGL((hc::k_crc_grp_perm<false, false>), dim3(cus), dim3(hc::kFastThreads), 0, st, b.base,
                           nullptr, nullptr, b.stride, b.ulen, 0u, N, lg, crc, nullptr, nullptr, dt, p, q);
    };
  };
  for (uint32_t lg : {7u, 5u}) {
    if (N & ((1u << lg) - 1)) continue;  // the permutation needs whole chunks
    const uint64_t q = N >> lg;
    char nm[128];
    std::snprintf(nm, sizeof nm, "identity C=%u (copy)", 1u << lg);
    vs.push_back({nm, perm(lg, 0, false), {}});
    const uint64_t p1 = coprime_near(q / cus, q), p2 = coprime_near((uint64_t)(q * 0.6180339887), q),
                   p3 = coprime_near(q / 8 + 1, q);
    std::snprintf(nm, sizeof nm, "perm C=%u p=%llu (~Q/G)", 1u << lg, (unsigned long long)p1);
    vs.push_back({nm, perm(lg, p1, false), {}});
    std::snprintf(nm, sizeof nm, "perm C=%u p=%llu (~0.618Q)", 1u << lg, (unsigned long long)p2);
    vs.push_back({nm, perm(lg, p2, false), {}});
    std::snprintf(nm, sizeof nm, "perm C=%u p=%llu (~Q/8) xcd", 1u << lg, (unsigned long long)p3);
    vs.push_back({nm, perm(lg, p3, true), {}});
  }
  vs.push_back({"PROD launch_grp (again)", [&](hipStream_t st) { CK(hc::launch_grp(b, cus, st)); }, {}});

  std::vector<uint32_t> ref(N), got(N);
  vs[0].run(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), crc, N * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto &v : vs) {
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
