// kany3.hip -- round-3 study of the general kernel (k_crc_any: any alignment,
// any length, whole messages).  The production kernel keeps 144 KiB of
// replicated LDS tables and 32 VGPRs of placement columns, so it runs one
// 16-wave workgroup per CU (VGPR- and LDS-bound alike) and measures 62-70 % of
// 8 TB/s, bound by its memory pattern: one wave per message, a round trip per
// 4-row batch.  k_crc_any_x (tools/gen_any_x.py: the product
// kernel copied at build time) uses the LDS-free row step and the workgroup-
// shared placement columns that lifted the framing kernels, and runs as 4-wave
// workgroups, several per CU: more waves in flight for a latency-bound pattern.
//
//   ./kany3 [nmsg=2000000] [rounds=5] [launches=5]
//
// Workloads: config 5b's record law with 16-B gaps (not packed: the stream
// does not take it), equal 9815-B records with gaps, 4092-B blocks via off/len
// in verify mode (stamped, every 997th corrupted), records of 16-1020 B (the
// lane mode).  Every variant's words (and verify bitmap / first bad) are
// checked against production's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "../hunddb_amd/csrc/hc_kernels.hip"
#include "build/k_crc_any_x.inc"

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
  std::function<void(const hc::Batch &, hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("device %s, %d CUs; %llu messages per workload\n", prop.gcnArchName, cus, (unsigned long long)N);
  hc::DeviceTables *dt;
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const uint64_t cap = 21ull << 30;
  uint8_t *buf;
  uint64_t *doff;
  uint32_t *dlen, *crc, *bm;
  unsigned long long *fb;
  CK(hipMalloc(&buf, cap));
  CK(hipMalloc(&doff, N * 8));
  CK(hipMalloc(&dlen, N * 4));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&bm, (N + 31) / 32 * 4));
  CK(hipMalloc(&fb, 8));

  std::vector<Variant> vs;
  vs.push_back({"PROD k_crc_any (16 waves, LDS tables)", [&](const hc::Batch &b, hipStream_t st) {
                  CK(hc::launch_general(b, 0, cus, st));
                }, {}});
#define XV(W, PER_CU, OCC)                                                                                        \
  vs.push_back({"X W=" #W " " #PER_CU "/CU occ>=" #OCC, [&](const hc::Batch &b, hipStream_t st) {                  \
                  const int g = cus * (PER_CU);                                                                   \
                  if (b.flags & hc::kFlagMessages)                                                                \
                    hipLaunchKernelGGL((hc::k_crc_any_x<true, W, OCC>), dim3(g), dim3((W) * 64), 0, st, b.base,   \
                                       b.off, b.len, b.stride, b.ulen, b.flags, b.nblocks, 0u, 0u, b.crc_out,     \
                                       b.bad_bitmap, b.first_bad, b.tables, nullptr);                             \
                  else                                                                                            \
                    hipLaunchKernelGGL((hc::k_crc_any_x<false, W, OCC>), dim3(g), dim3((W) * 64), 0, st, b.base,  \
                                       b.off, b.len, b.stride, b.ulen, b.flags, b.nblocks, 0u, 0u, b.crc_out,     \
                                       b.bad_bitmap, b.first_bad, b.tables, nullptr);                             \
                  CK(hipGetLastError());                                                                          \
                }, {}})
  XV(4, 4, 1);
  XV(4, 8, 1);
  XV(4, 16, 1);
  XV(8, 4, 1);
  XV(4, 8, 5);
  XV(4, 8, 6);

  struct Work {
    std::string name;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    bool msg;
  };
  std::vector<Work> works;
  {
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    Work a{"config 5b law, 16-B gaps (msg)", {}, {}, true}, e{"equal 9815 B, 7-B gaps (msg)", {}, {}, true},
        k{"4092-B blocks off/len, verify", {}, {}, false}, sm{"16-1020 B records, 16-B gaps (msg)", {}, {}, true};
    uint64_t pa = 1, pe = 3, pk = 0, ps = 5;
    for (uint64_t i = 0; i < N; i++) {
      const uint32_t la = (uint32_t)(64.0 * std::exp(U(rng) * std::log(1024.0)));
      a.off.push_back(pa), a.len.push_back(la), pa += la + 16;
      e.off.push_back(pe), e.len.push_back(9815), pe += 9815 + 7;
      k.off.push_back(pk), k.len.push_back(4092), pk += 4092;
      const uint32_t ls = 16 + (uint32_t)(U(rng) * 1004);
      sm.off.push_back(ps), sm.len.push_back(ls), ps += ls + 16;
    }
    works = {a, e, k, sm};
  }
  int bad = 0;
  for (auto &w : works) {
    const uint64_t span = w.off.back() + w.len.back() + 64;
    if (span > cap) {
      std::printf("skip %s: %llu bytes\n", w.name.c_str(), (unsigned long long)span);
      continue;
    }
    CK(hc::launch_fill(buf, nullptr, nullptr, 1 << 20, 1 << 20, (span + (1 << 20) - 1) >> 20, 0x4B41, cus * 16, s));
    CK(hipMemcpy(doff, w.off.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, w.len.data(), N * 4, hipMemcpyHostToDevice));
    hc::Batch b{};
    b.base = buf;
    b.off = doff;
    b.len = dlen;
    b.nblocks = N;
    b.tables = dt;
    b.crc_out = crc;
    uint64_t bytes = 0;
    for (auto l : w.len) bytes += l;
    if (!w.msg) {  // stamp every block, then corrupt every 997th
      hc::Batch st = b;
      st.flags = hc::kFlagStamp;
      st.crc_out = nullptr;
      CK(hc::launch_general(st, 0, cus, s));
      CK(hipStreamSynchronize(s));
      for (uint64_t i = 5; i < N; i += 997) CK(hipMemsetAsync(buf + w.off[i] + 100, 0x5A, 1, s));
      b.bad_bitmap = bm;
      b.first_bad = fb;
      bytes += 4 * N;
    } else {
      b.flags = hc::kFlagMessages;
      bytes += 4 * N;
    }
    auto prep = [&]() {
      if (!w.msg) CK(hc::launch_verify_prepare(bm, fb, N, s));
    };
    std::vector<uint32_t> ref(N), got(N), bref((N + 31) / 32), bgot(bref.size());
    unsigned long long fref = 0, fgot = 0;
    for (size_t v = 0; v < vs.size(); v++) {
      CK(hipMemsetAsync(crc, 0, N * 4, s));
      prep();
      vs[v].run(b, s);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(v == 0 ? ref.data() : got.data(), crc, N * 4, hipMemcpyDeviceToHost));
      if (!w.msg) {
        CK(hipMemcpy(v == 0 ? bref.data() : bgot.data(), bm, bref.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(v == 0 ? &fref : &fgot, fb, 8, hipMemcpyDeviceToHost));
      }
      if (v && (got != ref || (!w.msg && (bgot != bref || fgot != fref)))) {
        std::printf("MISMATCH %s / %s\n", w.name.c_str(), vs[v].name.c_str());
        bad++;
      }
    }
    for (auto &v : vs) v.ms.clear();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++)
      for (auto &v : vs)
        for (int l = 0; l < launches; l++) {
          prep();
          CK(hipEventRecord(e0, s));
          v.run(b, s);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          v.ms.push_back(ms);
        }
    std::printf("== %s: %.2f GB per launch\n", w.name.c_str(), bytes / 1e9);
    std::printf("%-40s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
    for (auto &v : vs) {
      std::sort(v.ms.begin(), v.ms.end());
      const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
      std::printf("%-40s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6,
                  bytes / med / 1e6 / 80.0, med);
    }
    std::fflush(stdout);
  }
  return bad ? 3 : 0;
}
