// kbench2.hip — A/B harness for k_crc_grp (per-workgroup block hand-out,
// chunked XCD-local block order) against the production kernels (one
// process, interleaved rounds, HIP-event time per launch).  Not part of the
// product; build: make -C tools kbench2.
//
//   ./kbench2 <mode> [nblocks=1000000] [rounds=8] [launches=5]
//   mode: 4096 | 8192 | 16384 (uniform batch) | mixed (configs[2]: 4/8/16 KiB
//         drawn as bench.py's mixed_sizes, packed, off/len) | offlen4k
//
// Every CRC variant's words are checked against the production output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "ab_hc_kernels.hip"
#include "ab_kernels.hip"
#include "r1_kernels.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

namespace {

uint64_t splitmix_h(uint64_t seed, uint64_t blk, uint64_t w) {
  uint64_t z = seed + ((blk << 21) + w) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Variant {
  std::string name;
  bool check;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

}  // namespace

int main(int argc, char **argv) {
  const std::string mode = argc > 1 ? argv[1] : "8192";
  const uint64_t N = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1000000;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 8;
  const int launches = argc > 4 ? std::atoi(argv[4]) : 5;
  // general-kernel modes (k_crc_any): msg = config 5b (log-uniform 64 B - 64 KiB
  // records packed back to back at an odd address, whole-message CRC), eq9815 =
  // equal 9815-B records, blk4092 = 4092-B blocks in block mode (off/len)
  // msgsmall / msgbig: the same log-uniform law restricted to records under /
  // at or over 1 KiB (what config 5b's small records cost)
  const bool logu = mode == "msg" || mode == "msgsmall" || mode == "msgbig";
  const bool general = logu || mode == "eq9815" || mode == "blk4092";
  const bool arrays = mode == "mixed" || mode == "offlen4k" || general;
  const uint32_t B = arrays ? 4096 : (uint32_t)std::atoi(mode.c_str());
  if (!arrays && (B == 0 || B % 4096 != 0)) {  // never launch a kernel outside its layout contract
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;

  std::vector<uint64_t> ho(N);
  std::vector<uint32_t> hl(N);
  uint64_t total = 0;
  if (general) total = 1;  // odd start
  for (uint64_t i = 0; i < N; i++) {
    uint32_t l = B;
    if (mode == "mixed") l = 4096u << (uint32_t)(splitmix_h(0x48756E64ull ^ 0x5A5A5A5A5A5A5A5Aull, i, (1u << 21) - 1) % 3);
    if (logu) {  // log-uniform in [64, 65536] (msgsmall: [64, 1024), msgbig: [1024, 65536])
      double u = (double)(splitmix_h(0x5B, i, 0) >> 11) / 9007199254740992.0;
      if (mode == "msgsmall") u *= 0.4;
      if (mode == "msgbig") u = 0.4 + 0.6 * u;
      l = (uint32_t)(64.0 * std::exp(u * std::log(1024.0)));
      if (mode == "msgsmall" && l >= 1024) l = 1023;
    }
    if (mode == "eq9815") l = 9815;
    if (mode == "blk4092") l = 4092;
    ho[i] = total;
    hl[i] = l;
    total += l;
  }
  total += 64;
  std::printf("device %s, %d CUs; mode %s: %llu blocks, %.3f GB\n", prop.gcnArchName, cus, mode.c_str(),
              (unsigned long long)N, total / 1e9);
  uint8_t *buf;
  uint32_t *crc, *crc_ref;
  uint64_t *doff;
  uint32_t *dlen;
  hc::DeviceTables *dt;
  CK(hipMalloc(&buf, total));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&crc_ref, N * 4));
  CK(hipMalloc(&doff, N * 8));
  CK(hipMalloc(&dlen, N * 4));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  CK(hipMemcpy(doff, ho.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlen, hl.data(), N * 4, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hc::launch_fill(buf, doff, dlen, 0, 0, N, 0x48756E64, cus * 16, s));
  CK(hipStreamSynchronize(s));

  hc::Batch b{};
  b.base = buf;
  b.stride = B;
  b.ulen = B;
  b.nblocks = N;
  b.tables = dt;
  if (arrays) {
    b.off = doff;
    b.len = dlen;
  }
  if (logu || mode == "eq9815") b.flags = hc::kFlagMessages;
  hc::SegTables *seg_t;
  CK(hipMalloc(&seg_t, sizeof(hc::SegTables)));
  {
    std::vector<hc::SegTables> h(1);
    hc::build_seg_tables(h[0]);
    CK(hipMemcpy(seg_t, h.data(), sizeof(hc::SegTables), hipMemcpyHostToDevice));
  }
  const uint64_t seg_mu = hc::seg_max_units(total + 1024);
  uint32_t *seg_ws;
  CK(hipMalloc(&seg_ws, hc::seg_workspace_bytes(N, seg_mu)));
  const uint32_t lg5 = 5;
  using namespace hc;
  std::vector<Variant> vs;
  auto add = [&](const char *name, bool check, std::function<void(hipStream_t)> f) {
    vs.push_back(Variant{name, check, f, {}});
  };
#define GRP(ARR, DYN, NUL, LG, ...)                                                                                   \
  [&](hipStream_t st) {                                                                                          \
    hipLaunchKernelGGL((k_crc_grp<ARR, DYN, NUL __VA_OPT__(,) __VA_ARGS__>), dim3(cus), dim3(kFastThreads), 0, st, b.base, b.off, b.len,  \
                       b.stride, b.ulen, b.flags, b.nblocks, (uint32_t)(LG), b.crc_out, b.bad_bitmap, b.first_bad, \
                       b.tables);                                                                                \
  }
  // chunk sweep: HC_SWEEP=1 times k_crc_grp at lg_chunk 3..8 (C = 8 .. 256)
  const bool sweep = std::getenv("HC_SWEEP") != nullptr;
  if (general) {
    add("r1 k_crc_any static runs", true, [&](hipStream_t st) { launch_general_static(b, 0, cus, st); });
    add("k_crc_any dyn C=1 window", true, [&](hipStream_t st) { launch_general_dyn(b, 0, cus, st, 0); });
    add("k_crc_any dyn C=2 windows", true, [&](hipStream_t st) { launch_general_dyn(b, 0, cus, st, 1); });
    add("k_crc_any dyn C=4 windows", true, [&](hipStream_t st) { launch_general_dyn(b, 0, cus, st, 2); });
    add("k_crc_any dyn C=16 windows", true, [&](hipStream_t st) { launch_general_dyn(b, 0, cus, st, 4); });
    add("r1 static (again)", true, [&](hipStream_t st) { launch_general_static(b, 0, cus, st); });
    add("PROD launch_general (dyn, 1 window)", true, [&](hipStream_t st) { launch_general(b, 0, cus, st); });
    add("k_crc_any dyn C=4 (again)", true, [&](hipStream_t st) { launch_general_dyn(b, 0, cus, st, 2); });
#define ANYV(BATCH, VAR)                                                                                        \
  [&](hipStream_t st) {                                                                                         \
    hipLaunchKernelGGL((k_crc_any<BATCH, VAR, true>), dim3(cus), dim3(kFastThreads), 0, st, b.base, b.off, b.len, \
                       b.stride, b.ulen, b.flags, b.nblocks, 0u, 0u, b.crc_out, b.bad_bitmap, b.first_bad, b.tables); \
  }
    if (b.flags & kFlagMessages) {  // packed records: one stream over the span (k_seg_*)
      add("SEG packed stream (6 launches)", true, [&](hipStream_t st) { launch_seg(b, seg_t, seg_ws, seg_mu, cus, st); });
#define SEGSTREAM(NUL, NOEV, LG)                                                                               \
  [&](hipStream_t st) {                                                                                       \
    hipLaunchKernelGGL((k_seg_stream<NUL, NOEV>), dim3(cus), dim3(kFastThreads), 0, st, b.base, b.off, b.len,  \
                       b.nblocks, (uint32_t)(LG), seg_ws, seg_ws + 64, seg_ws + 64 + seg_mu + 1,                  \
                       seg_ws + 64 + 3 * seg_mu + 1 + 2 * ((seg_mu >> 10) + 1), b.tables);                         \
  }
      add("SEG k_seg_stream alone (C=128)", false, SEGSTREAM(false, false, 7));
      add("SEG k_seg_stream NULL math", false, SEGSTREAM(true, false, 7));
      add("SEG k_seg_stream no events", false, SEGSTREAM(false, true, 7));
      add("SEG k_seg_stream NULL + no events", false, SEGSTREAM(true, true, 7));
      if (sweep) {
        add("SEG packed stream C=8", true, [&](hipStream_t st) { launch_seg(b, seg_t, seg_ws, seg_mu, cus, st, nullptr, 3); });
        add("SEG packed stream C=16", true, [&](hipStream_t st) { launch_seg(b, seg_t, seg_ws, seg_mu, cus, st, nullptr, 4); });
        add("SEG packed stream C=32", true, [&](hipStream_t st) { launch_seg(b, seg_t, seg_ws, seg_mu, cus, st, nullptr, 5); });
        add("SEG packed stream C=64", true, [&](hipStream_t st) { launch_seg(b, seg_t, seg_ws, seg_mu, cus, st, nullptr, 6); });
        add("SEG k_seg_stream NULL+noev C=8", false, SEGSTREAM(true, true, 3));
        add("SEG k_seg_stream NULL+noev C=16", false, SEGSTREAM(true, true, 4));
        add("SEG k_seg_stream NULL+noev C=32", false, SEGSTREAM(true, true, 5));
      }
      add("SEG packed stream (again)", true, [&](hipStream_t st) { launch_seg(b, seg_t, seg_ws, seg_mu, cus, st); });
    }
    add("PROD launch_general (again)", true, [&](hipStream_t st) { launch_general(b, 0, cus, st); });
  } else if (!arrays) {
    add("PROD k_crc_uni", true, [&](hipStream_t st) { launch_uni(b, cus, st); });
    if (sweep) {
      add("grp pinned C=8", true, GRP(false, true, false, 3, true));
      add("grp pinned C=16", true, GRP(false, true, false, 4, true));
      add("grp pinned C=32", true, GRP(false, true, false, 5, true));
      add("grp pinned C=64", true, GRP(false, true, false, 6, true));
      add("grp pinned C=128", true, GRP(false, true, false, 7, true));
      add("grp pinned C=256", true, GRP(false, true, false, 8, true));
      add("grp pinned C=512", true, GRP(false, true, false, 9, true));
      add("production launch_grp", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
    } else if (std::getenv("KB2_PIECE") && (B == 8192 || B == 16384)) {  // 4 KiB pieces of 8/16 KiB blocks
#define PIECE(GG, LG, X)                                                                                      \
  [&](hipStream_t st) {                                                                                      \
    hipLaunchKernelGGL((k_crc_piece<GG, X>), dim3(cus), dim3(kFastThreads), 0, st, b.base, b.stride, b.flags,  \
                       b.nblocks, (uint32_t)(LG), b.crc_out, b.bad_bitmap, b.first_bad, b.tables, seg_t);       \
  }
      add("PROD launch_grp", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
      if (B == 8192) {
        add("PIECE G=2 C=64 pieces", true, PIECE(2, 6, false));
        add("PIECE G=2 C=32 pieces", true, PIECE(2, 5, false));
        add("PIECE G=2 C=128 pieces", true, PIECE(2, 7, false));
        add("PIECE G=2 XCD C=64 pieces", true, PIECE(2, 6, true));
        add("PIECE G=2 XCD C=32 pieces", true, PIECE(2, 5, true));
      } else {
        add("PIECE G=4 C=64 pieces", true, PIECE(4, 6, false));
        add("PIECE G=4 C=128 pieces", true, PIECE(4, 7, false));
        add("PIECE G=4 XCD C=64 pieces", true, PIECE(4, 6, true));
      }
      add("PROD launch_grp (again)", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
    } else {
      add("PROD launch_grp", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
      if (std::getenv("KB2_NIB")) {  // nibble shift4 tables (conflict-free finalise)
        if (B >= 8192) {
          add("NIB grp XCD C=32", true, GRP(false, true, false, 5, true, false, true, true));
          add("PROD launch_grp (2)", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
          add("NIB grp XCD C=32 (2)", true, GRP(false, true, false, 5, true, false, true, true));
        } else {
          add("NIB grp C=64", true, GRP(false, true, false, 6, true, false, false, true));
          add("PROD launch_grp (2)", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
          add("NIB grp C=64 (2)", true, GRP(false, true, false, 6, true, false, false, true));
        }
      }
      add("grp pinned C=64", true, GRP(false, true, false, 6, true));
      add("grp pinned C=128", true, GRP(false, true, false, 7, true));
      add("grp XCD-contiguous C=16", true, GRP(false, true, false, 4, true, false, true));
      add("grp XCD-contiguous C=32", true, GRP(false, true, false, 5, true, false, true));
      add("grp XCD-contiguous C=64", true, GRP(false, true, false, 6, true, false, true));
      add("grp XCD-contiguous C=128", true, GRP(false, true, false, 7, true, false, true));
      add("PROD launch_grp (again)", true, [&](hipStream_t st) { launch_grp(b, cus, st); });
      add("grp pinned C=128 (round-2 r1 production at 8/16 KiB)", true, GRP(false, true, false, 7, true));
    }
  } else {
    add("r1 k_crc_fast + k_crc_any(1023)", true, [&](hipStream_t st) {
      launch_fast(b, false, cus, st);
      launch_general_static(b, 1023, cus, st);
    });
#define GRPANY(LG)                             \
  [&](hipStream_t st) {                     \
    GRP(true, true, false, LG, true)(st);      \
    launch_general(b, 4095, cus, st);       \
  }
    if (sweep) {
      add("grp pinned C=8 + any(4095)", true, GRPANY(3));
      add("grp pinned C=16 + any(4095)", true, GRPANY(4));
      add("grp pinned C=32 + any(4095)", true, GRPANY(5));
      add("grp pinned C=64 + any(4095)", true, GRPANY(6));
      add("grp pinned C=128 + any(4095)", true, GRPANY(7));
      add("grp pinned C=256 + any(4095)", true, GRPANY(8));
      add("production launch_grp + any", true, [&](hipStream_t st) {
        launch_grp(b, cus, st);
        launch_general(b, 4095, cus, st);
      });
    } else {
      add("PROD launch_grp + any", true, [&](hipStream_t st) {
        launch_grp(b, cus, st);
        launch_general(b, 4095, cus, st);
      });
      add("grp BATCH refill C=64 + any", true, [&](hipStream_t st) {
        GRP(true, true, false, 6, false, true)(st);
        launch_general(b, 4095, cus, st);
      });
      add("grp pinned C=64 + any(4095)", true, GRPANY(6));
      add("NULL grp pinned C=64", false, GRP(true, true, true, 6, true));
      add("NULL grp BATCH C=64", false, GRP(true, true, true, 6, false, true));
      add("PROD launch_grp + any (again)", true, [&](hipStream_t st) {
        launch_grp(b, cus, st);
        launch_general(b, 4095, cus, st);
      });
    }
  }

  b.crc_out = crc_ref;
  vs[0].run(s);
  CK(hipStreamSynchronize(s));
  std::vector<uint32_t> ref(N), got(N);
  CK(hipMemcpy(ref.data(), crc_ref, N * 4, hipMemcpyDeviceToHost));
  b.crc_out = crc;
  int bad = 0;
  for (auto &v : vs) {
    if (v.check) {
      CK(hipMemsetAsync(crc, 0, N * 4, s));
      v.run(s);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(got.data(), crc, N * 4, hipMemcpyDeviceToHost));
      if (got != ref) {
        uint64_t k = 0;
        while (k < N && got[k] == ref[k]) k++;
        std::printf("MISMATCH in variant %s at block %llu (%08x vs %08x)\n", v.name.c_str(), (unsigned long long)k,
                    got[k], ref[k]);
        bad++;
      }
    } else {
      v.run(s);
    }
  }
  CK(hipStreamSynchronize(s));
  if (b.flags & kFlagMessages) {
    uint32_t fl = 0;
    CK(hipMemcpy(&fl, seg_ws, 4, hipMemcpyDeviceToHost));
    std::printf("seg flag (1 = not taken) = %u\n", fl);
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
  std::printf("%-40s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-40s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), total / med / 1e6, total / best / 1e6,
                total / med / 1e6 / 80.0, med);
  }
  return bad ? 3 : 0;
}
