// kframe.hip — A/B harness for the read+write framing kernels (k_frame = fused
// AddCRCsToData, k_unframe = batched ReadFromDisk): blocks in flight per wave
// (2 or 3), chunk size of the per-CU hand-out, and timing-only (XOR) builds
// that isolate the memory pattern.  One process, interleaved rounds, HIP-event
// time per launch.  Not part of the product; build: make -C tools kframe.
//
//   ./kframe [nblocks=1000000] [rounds=6] [launches=5]
//
// GB/s = bytes read + bytes written per launch / launch time.  Every CRC
// variant's output bytes and CRC words are checked against the production
// configuration's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "ab_hc_kernels.hip"
#include "ab_kernels.hip"

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
  int kind;  // 0 frame, 1 unframe
  bool check;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint64_t npay = N * 4092 - 1000;  // ragged last block, as bench.py --workload frame
  std::printf("device %s, %d CUs; %llu blocks (frame: %llu B payload at an odd address)\n", prop.gcnArchName, cus,
              (unsigned long long)N, (unsigned long long)npay);
  uint8_t *raw, *framed, *framed_ref, *blocks, *pay, *pay_ref;
  uint32_t *crc, *crc_ref, *bitmap;
  unsigned long long *fb;
  hc::DeviceTables *dt;
  // KFRAME_ORDER=bench: the unframe buffers first, in bench.py's order (blocks,
  // payload); the HBM placement of the two streams moves k_unframe by ~2 %
  if (std::getenv("KFRAME_ORDER")) {
    CK(hipMalloc(&blocks, N * 4096));
    CK(hipMalloc(&pay, N * 4092));
  }
  CK(hipMalloc(&raw, npay + 16));
  CK(hipMalloc(&framed, N * 4096));
  CK(hipMalloc(&framed_ref, N * 4096));
  if (!std::getenv("KFRAME_ORDER")) {
    CK(hipMalloc(&blocks, N * 4096));
    CK(hipMalloc(&pay, N * 4092));
  }
  CK(hipMalloc(&pay_ref, N * 4092));
  std::printf("blocks %p payload %p\n", (void *)blocks, (void *)pay);
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&crc_ref, N * 4));
  CK(hipMalloc(&bitmap, (N + 31) / 32 * 4));
  CK(hipMalloc(&fb, 8));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const uint8_t *src = raw + 1;
  CK(hc::launch_fill(raw, nullptr, nullptr, npay + 16, npay + 16, 1, 0x48756E64, cus * 16, s));
  CK(hc::launch_fill(blocks, nullptr, nullptr, 4096, 4096, N, 0x5EED, cus * 16, s));
  {  // stamp the unframe input
    hc::Batch b{};
    b.base = blocks;
    b.stride = 4096;
    b.ulen = 4096;
    b.nblocks = N;
    b.flags = hc::kFlagStamp;
    b.tables = dt;
    CK(hc::launch_grp(b, cus, s));
  }
  CK(hc::launch_verify_prepare(bitmap, fb, N, s));
  CK(hipStreamSynchronize(s));
  const uint64_t nblk = N, ni = nblk - 2;
  using namespace hc;
  std::vector<Variant> vs;
#define FRAME(D, NUL, LG, ...)                                                                                     \
  [&, lg = (uint32_t)(LG)](hipStream_t st) {                                                                        \
    hipLaunchKernelGGL((k_frame<D, NUL __VA_OPT__(,) __VA_ARGS__>), dim3(cus), dim3(kFastThreads), 0, st, src, npay, \
                       framed, nblk, lg, crc, dt);                                                                  \
  }
#define FRAME_NP(R, PER)                                                                                         \
  [&](hipStream_t st) {                                                                                          \
    const uint64_t g_ = (ni + 4 * (PER)-1) / (4 * (PER));                                                         \
    hipLaunchKernelGGL((k_frame_np<R, PER>), dim3((unsigned)(g_ ? g_ : 1)), dim3(256), 0, st, src, npay, framed, nblk, \
                       crc, dt);                                                                                 \
  }
#define UNFRAME(D, NUL, LG, ...)                                                                                   \
  [&, lg = (uint32_t)(LG)](hipStream_t st) {                                                                        \
    hipLaunchKernelGGL((k_unframe<0, D, NUL __VA_OPT__(,) __VA_ARGS__>), dim3(cus), dim3(kFastThreads), 0, st, blocks, \
                       nblk, lg, pay, crc, bitmap, fb, dt);                                                         \
  }
  const uint32_t lgp = grp_lg_chunk(ni, cus, 4096);
  vs.push_back({"PROD k_frame depth 2", 0, true, FRAME(2, false, lgp), {}});
  if (std::getenv("KFRAME_XCD")) {
    vs.push_back({"k_frame XCD C=16", 0, true, FRAME(2, false, 4, true), {}});
    vs.push_back({"k_frame XCD C=32", 0, true, FRAME(2, false, 5, true), {}});
  }
  vs.push_back({"np frame R=4 1 blk/wave", 0, true, FRAME_NP(4, 1), {}});
  vs.push_back({"np frame R=4 2 blk/wave", 0, true, FRAME_NP(4, 2), {}});
  vs.push_back({"np frame R=8 1 blk/wave", 0, true, FRAME_NP(8, 1), {}});
  vs.push_back({"np frame R=2 1 blk/wave", 0, true, FRAME_NP(2, 1), {}});
  vs.push_back({"np frame R=4 4 blk/wave", 0, true, FRAME_NP(4, 4), {}});
  vs.push_back({"k_frame hash then 4 stores", 0, true, FRAME(2, false, lgp, false, 2), {}});
  vs.push_back({"k_frame 4 stores then hash", 0, true, FRAME(2, false, lgp, false, 4), {}});
  vs.push_back({"NULL k_frame", 0, false, FRAME(2, true, lgp), {}});
  vs.push_back({"NULL k_frame hash then 4 stores", 0, false, FRAME(2, true, lgp, false, 2), {}});
  vs.push_back({"PROD k_unframe depth 2", 1, true, UNFRAME(2, false, lgp), {}});
  vs.push_back({"k_unframe round-2 store order (each row, then hash)", 1, true, UNFRAME(2, false, lgp, false, 0), {}});
  vs.push_back({"k_unframe buffer stores nt", 1, true, UNFRAME(2, false, lgp, false, 2, 3), {}});
  vs.push_back({"k_unframe buffer stores sc0|nt", 1, true, UNFRAME(2, false, lgp, false, 2, 4), {}});
  vs.push_back({"k_unframe buffer stores sc1|nt", 1, true, UNFRAME(2, false, lgp, false, 2, 19), {}});
  vs.push_back({"k_unframe buffer stores sc0|sc1|nt", 1, true, UNFRAME(2, false, lgp, false, 2, 20), {}});
  vs.push_back({"k_unframe buffer stores sc1", 1, true, UNFRAME(2, false, lgp, false, 2, 17), {}});
  vs.push_back({"k_unframe stores after rows 0-2", 1, true, UNFRAME(2, false, lgp, false, 4), {}});
  vs.push_back({"NULL k_unframe 4 stores after group", 1, false, UNFRAME(2, true, lgp, false, 2), {}});
  vs.push_back({"k_unframe 4 stores after group, depth 3", 1, true, UNFRAME(3, false, lgp, false, 2), {}});
  vs.push_back({"NULL k_unframe round-2 order", 1, false, UNFRAME(2, true, lgp, false, 0), {}});
  vs.push_back({"k_unframe store after hash", 1, true, UNFRAME(2, false, lgp, false, 1), {}});
  vs.push_back({"k_unframe 4 stores after group", 1, true, UNFRAME(2, false, lgp, false, 2), {}});
  vs.push_back({"k_unframe write-back stores", 1, true, UNFRAME(2, false, lgp, false, 3), {}});
  vs.push_back({"NULL k_unframe write-back stores", 1, false, UNFRAME(2, true, lgp, false, 3), {}});
  vs.push_back({"NULL k_unframe (production order)", 1, false, UNFRAME(2, true, lgp), {}});
  vs.push_back({"PROD k_frame depth 2 (again)", 0, true, FRAME(2, false, lgp), {}});
  vs.push_back({"PROD k_unframe depth 2 (again)", 1, true, UNFRAME(2, false, lgp), {}});

  // reference outputs
  std::vector<uint32_t> cref_f(N), cref_u(N), got(N);
  vs[0].run(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(framed_ref, framed, N * 4096, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(cref_f.data(), crc, N * 4, hipMemcpyDeviceToHost));
  for (auto &v : vs)
    if (v.kind == 1) {  // PROD k_unframe
      v.run(s);
      break;
    }
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(pay_ref, pay, N * 4092, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(cref_u.data(), crc, N * 4, hipMemcpyDeviceToHost));
  std::vector<uint8_t> h1, h2;
  int bad = 0;
  for (auto &v : vs) {
    if (!v.check) {
      v.run(s);
      continue;
    }
    CK(hipMemsetAsync(crc, 0, N * 4, s));
    CK(hipMemsetAsync(v.kind ? pay : framed, 0x77, v.kind ? N * 4092 : N * 4096, s));
    v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), crc, N * 4, hipMemcpyDeviceToHost));
    const size_t bytes = v.kind ? N * 4092 : N * 4096;
    h1.resize(bytes);
    h2.resize(bytes);
    CK(hipMemcpy(h1.data(), v.kind ? pay : framed, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), v.kind ? pay_ref : framed_ref, bytes, hipMemcpyDeviceToHost));
    if (got != (v.kind ? cref_u : cref_f) || h1 != h2) {
      std::printf("MISMATCH in variant %s\n", v.name.c_str());
      bad++;
    }
  }
  CK(hipStreamSynchronize(s));
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
  std::printf("%-36s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double bytes = v.kind ? (double)N * (4096 + 4092) : (double)npay + N * 4096.0;
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-36s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6,
                bytes / med / 1e6 / 80.0, med);
  }
  return bad ? 3 : 0;
}
