// kcopy.hip — memory-pattern A/B harness for the read+write kernels (k_frame,
// k_unframe).  Not part of the product; build: make -C tools kcopy.
//
//   ./kcopy [nchunks=1000000] [rounds=6] [launches=5]
//
// Every variant moves nchunks 4 KiB chunks (1024 B rows, 16 B per lane) from
// src to dst and XOR-folds what it read (no CRC), so it measures only the
// memory pattern.  "frame" geometry: src chunk c at src + 4092c - 4 + 1 (odd,
// unaligned, like k_frame's payload), dst chunk at 4096c.  "unframe": src at
// 4096c (aligned), dst at 4092c - 4 (unaligned).  Also: the production k_frame
// and k_unframe, and plain grid-stride uint4 copies.  GB/s = read + written
// bytes / HIP-event launch time (median over interleaved rounds).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "ab_hc_kernels.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

namespace {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

template <int kPol>
__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
  if constexpr (kPol == 1) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(p));
  return *reinterpret_cast<const u32x4_u *>(p);
}
template <int kPol>
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) {
  if constexpr (kPol == 1)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4_u *>(p));
  else
    *reinterpret_cast<u32x4_u *>(p) = v;
}

// Chunk pattern: kDepth chunks per wave in a register ring (kDepth-1 in flight
// while one is stored); kOrder 0 = each wave owns a contiguous run of chunks,
// 1 = chunk c goes to wave c % W (neighbouring waves touch neighbouring chunks).
template <int kWaves, int kDepth, int kOrder, int kLd, int kSt, int kLdsKiB>
__global__ __launch_bounds__(kWaves * 64) void k_pat(const uint8_t *src, int64_t ss, int64_t so, uint8_t *dst,
                                                     int64_t ds, int64_t dso, uint64_t n, uint32_t *sink) {
  // occupancy as in the product kernels (kLdsKiB of LDS per workgroup)
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + hc::uni(threadIdx.x >> 6);
  const uint64_t W = (uint64_t)gridDim.x * kWaves;
  uint64_t c0, c1, step;
  if constexpr (kOrder == 0) {
    c0 = hc::uni64(n * gw / W);
    c1 = hc::uni64(n * (gw + 1) / W);
    step = 1;
  } else {
    c0 = gw;
    c1 = n;
    step = W;
  }
  if (c0 >= c1) return;
  const uint64_t last = c0 + (c1 - 1 - c0) / step * step;
  u32x4 R[kDepth][4];
  auto load = [&](uint64_t c, u32x4 (&v)[4]) {
    c = c < last ? c : last;
    const uint8_t *S = src + (int64_t)c * ss + so + 16 * lane;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = ld<kLd>(S + r * 1024);
  };
  uint32_t acc = 0;
#pragma unroll
  for (int d = 0; d < kDepth; d++) load(c0 + d * step, R[d]);
  for (uint64_t c = c0;;) {
#pragma unroll
    for (int d = 0; d < kDepth; d++) {
      uint8_t *D = dst + (int64_t)c * ds + dso + 16 * lane;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        st<kSt>(D + r * 1024, R[d][r]);
        acc ^= R[d][r].x ^ R[d][r].w;
      }
      load(c + kDepth * step, R[d]);
      c += step;
      if (c >= c1) {
        if (acc == 0x12345678u) sink[0] = acc + lds_pad[lane];
        return;
      }
    }
  }
}

template <int kLd, int kSt>
__global__ __launch_bounds__(256) void k_gscopy(const uint8_t *src, uint8_t *dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 a = ld<kLd>(src + 16 * i), b = ld<kLd>(src + 16 * (i + stride)), c = ld<kLd>(src + 16 * (i + 2 * stride)),
          d = ld<kLd>(src + 16 * (i + 3 * stride));
    st<kSt>(dst + 16 * i, a);
    st<kSt>(dst + 16 * (i + stride), b);
    st<kSt>(dst + 16 * (i + 2 * stride), c);
    st<kSt>(dst + 16 * (i + 3 * stride), d);
  }
  for (; i < n16; i += stride) st<kSt>(dst + 16 * i, ld<kLd>(src + 16 * i));
}

struct Variant {
  std::string name;
  double bytes;
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
  std::printf("device %s (%s), %d CUs; %llu chunks of 4 KiB\n", prop.name, prop.gcnArchName, cus,
              (unsigned long long)N);
  uint8_t *a, *b;
  uint32_t *sink, *crc, *bm;
  unsigned long long *fb;
  hc::DeviceTables *dt;
  const size_t bytes = N * 4096 + 4096;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(sink, 0, 4096));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&bm, N / 8 + 64));
  CK(hipMalloc(&fb, 8));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hc::launch_fill(a, nullptr, nullptr, bytes, bytes, 1, 7, cus * 16, s));
  CK(hc::launch_fill(b, nullptr, nullptr, bytes, bytes, 1, 9, cus * 16, s));
  {  // stamp the unframe source blocks (a clean verify pass)
    hc::Batch sb{};
    sb.base = a;
    sb.stride = 4096;
    sb.ulen = 4096;
    sb.nblocks = N;
    sb.flags = hc::kFlagStamp;
    sb.tables = dt;
    CK(hc::launch_fast(sb, true, cus, s));
    CK(hc::launch_verify_prepare(bm, fb, N, s));
  }
  const double fr = (double)N * 4092 + (double)N * 4096;  // frame/unframe bytes
  const uint8_t *fsrc = a + 4096 + 1;                        // frame payload (odd address)
  uint8_t *fdst = b;
  const uint8_t *usrc = a;        // unframe blocks
  uint8_t *udst = b + 4096;       // unframe payload
  std::vector<Variant> vs;
  constexpr int kLds = 144;
#define PAT(NAME, WV, DEP, ORD, LP, SP, GRIDMUL, LDSB, FRAME)                                                  \
  vs.push_back({NAME, fr, [=](hipStream_t st) {                                                                 \
                  auto k = k_pat<WV, DEP, ORD, LP, SP, LDSB>;                                                         \
                  if (FRAME)                                                                                    \
                    hipLaunchKernelGGL(k, dim3(cus * GRIDMUL), dim3(WV * 64), 0, st, fsrc, 4092, -4, fdst,   \
                                       4096, 0, N, sink);                                                       \
                  else                                                                                          \
                    hipLaunchKernelGGL(k, dim3(cus * GRIDMUL), dim3(WV * 64), 0, st, usrc, 4096, 0, udst, \
                                       4092, -4, N, sink);                                                      \
                }})
  vs.push_back({"PROD k_frame (inter)", fr, [=](hipStream_t st) { hc::launch_frame(fsrc, N * 4092, fdst, crc, dt, cus, st); }});
  vs.push_back({"k_frame contig", fr, [=](hipStream_t st) {
                  hipLaunchKernelGGL(hc::k_frame<false>, dim3(cus), dim3(hc::kFastThreads), 0, st, fsrc,
                                     (uint64_t)N * 4092, fdst, N, crc, dt);
                }});
  vs.push_back({"PROD k_unframe", fr, [=](hipStream_t st) {
                  hc::launch_unframe(usrc, N, 0, udst, crc, bm, fb, dt, cus, st);
                }});
  PAT("frame pat w16 d2 contig nt/nt (=k_frame)", 16, 2, 0, 1, 1, 1, kLds, true);
  PAT("frame pat w16 d3 contig nt/nt", 16, 3, 0, 1, 1, 1, kLds, true);
  PAT("frame pat w16 d2 inter nt/nt", 16, 2, 1, 1, 1, 1, kLds, true);
  PAT("frame pat w16 d3 inter nt/nt", 16, 3, 1, 1, 1, 1, kLds, true);
  PAT("frame pat w16 d2 contig pl/pl", 16, 2, 0, 0, 0, 1, kLds, true);
  PAT("frame pat w16 d2 inter pl/pl", 16, 2, 1, 0, 0, 1, kLds, true);
  PAT("frame pat w16 d2 inter nt/pl", 16, 2, 1, 1, 0, 1, kLds, true);
  PAT("frame pat w16 d2 contig nt/nt noLDS 2/CU", 16, 2, 0, 1, 1, 2, 0, true);
  PAT("frame pat w16 d2 inter nt/nt noLDS 2/CU", 16, 2, 1, 1, 1, 2, 0, true);
  PAT("frame pat w8 d2 inter nt/nt noLDS 4/CU", 8, 2, 1, 1, 1, 4, 0, true);
  PAT("unframe pat w16 d2 contig nt/nt (=k_unframe)", 16, 2, 0, 1, 1, 1, kLds, false);
  PAT("unframe pat w16 d3 contig nt/nt", 16, 3, 0, 1, 1, 1, kLds, false);
  PAT("unframe pat w16 d2 inter nt/nt", 16, 2, 1, 1, 1, 1, kLds, false);
  PAT("unframe pat w16 d3 inter nt/nt", 16, 3, 1, 1, 1, 1, kLds, false);
  PAT("unframe pat w16 d2 inter pl/pl", 16, 2, 1, 0, 0, 1, kLds, false);
  for (int v = 0; v < 4; v++) {
    const char *nm[] = {"gs copy pl/pl aligned", "gs copy nt/nt aligned", "gs copy nt/pl aligned",
                        "gs copy pl/nt aligned"};
    const size_t n16 = N * 4092 / 16;
    vs.push_back({nm[v], 2.0 * n16 * 16, [=](hipStream_t st) {
                    if (v == 0) hipLaunchKernelGGL((k_gscopy<0, 0>), dim3(cus * 8), dim3(256), 0, st, a, b, n16);
                    if (v == 1) hipLaunchKernelGGL((k_gscopy<1, 1>), dim3(cus * 8), dim3(256), 0, st, a, b, n16);
                    if (v == 2) hipLaunchKernelGGL((k_gscopy<1, 0>), dim3(cus * 8), dim3(256), 0, st, a, b, n16);
                    if (v == 3) hipLaunchKernelGGL((k_gscopy<0, 1>), dim3(cus * 8), dim3(256), 0, st, a, b, n16);
                  }});
  }
  for (auto &v : vs) v.run(s);  // warm
  CK(hipStreamSynchronize(s));
  CK(hipGetLastError());
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
  std::printf("%-48s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-48s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), v.bytes / med / 1e6, v.bytes / best / 1e6,
                v.bytes / med / 1e6 / 80.0, med);
  }
  return 0;
}
