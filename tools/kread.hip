// kread.hip — the read-stream ceiling of this chip: persistent (k_crc_grp's
// geometry and hand-out) against non-persistent grids.  Not part of the
// product; build: make -C tools kread.
//
//   ./kread [MiB=8192] [rounds=6] [launches=5]
//
// GB/s = bytes read / HIP-event launch time, median over interleaved rounds.
// Every variant XOR-folds what it reads into one word per wave (kept live by
// a never-true store), so no load is dead.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

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

template <int kNt>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (kNt) return __builtin_nontemporal_load(p);
  return *p;
}

__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// non-persistent: a workgroup of kWaves waves; wave w reads kPer consecutive
// 1 KiB rows (all loads issued before the first use), then exits.  kLdsKiB
// pads the workgroup's LDS like the CRC kernels (occupancy).
template <int kWaves, int kPer, int kLdsKiB, int kNt>
__global__ __launch_bounds__(kWaves * 64) void k_npread(const uint8_t *__restrict__ src, uint64_t nrows,
                                                        uint32_t *sink) {
  __shared__ uint32_t lds_pad[kLdsKiB * 256 + 1];
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t r0 = ((uint64_t)blockIdx.x * kWaves + wave) * kPer;
  if (r0 >= nrows) return;
  const u32x4 *S = reinterpret_cast<const u32x4 *>(src + r0 * 1024) + lane;
  u32x4 v[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) v[r] = ld<kNt>(S + r * 64);
  uint32_t acc = 0;
#pragma unroll
  for (int r = 0; r < kPer; r++) acc ^= fold(v[r]);
  if (acc == 0x12345679u) sink[0] = acc;
}

// k_crc_grp's pattern without the arithmetic: one 1024-thread workgroup per CU
// with 144 KiB of LDS, per-CU chunks of 2^kLg pieces of kRows 1 KiB rows handed
// out one at a time from an LDS counter, 4 rows in flight per wave with
// rolling refills (row r+4 issued right after row r is consumed).
template <int kRows, int kLg>
__global__ __launch_bounds__(1024) void k_dynread(const uint8_t *__restrict__ src, uint64_t npieces, uint32_t *sink) {
  __shared__ uint32_t lds_pad[144 * 256 + 1];
  __shared__ uint32_t ctr;
  if (threadIdx.x == 0) ctr = 16;
  if (sink[1] == 0xDEADu) lds_pad[threadIdx.x] = 1;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t G = gridDim.x, g = blockIdx.x;
  auto piece = [&](uint32_t k) -> uint64_t {
    return (((uint64_t)(k >> kLg) * G + g) << kLg) | (k & ((1u << kLg) - 1u));
  };
  uint64_t p = piece(wave);
  if (p >= npieces) return;
  uint32_t knv = 0;
  if (lane == 0) knv = atomicAdd(&ctr, 1u);
  // row stream of this wave: rows of piece p, then of the next handed-out piece
  uint64_t np = piece(__builtin_amdgcn_readfirstlane(knv));
  if (lane == 0) knv = atomicAdd(&ctr, 1u);
  u32x4 R[4];
  const u32x4 *S = reinterpret_cast<const u32x4 *>(src) + lane;
  uint64_t lastv = p;
  auto rowaddr = [&](uint64_t pc, int r) { return S + (pc * kRows + r) * 64; };
#pragma unroll
  for (int r = 0; r < 4; r++) R[r] = __builtin_nontemporal_load(rowaddr(p, r % kRows + 0 * r));
  uint32_t acc = 0;
  for (;;) {
    // consume piece p's rows; refill each slot with the row 4 ahead in the stream
#pragma unroll
    for (int r = 0; r < kRows; r++) {
      acc ^= fold(R[r & 3]);
      const int ahead = r + 4;
      const uint64_t pc = ahead < kRows ? p : (np < npieces ? np : lastv);
      const int rr = ahead < kRows ? ahead : ahead - kRows;
      R[r & 3] = __builtin_nontemporal_load(rowaddr(pc, rr));
    }
    if (np >= npieces) break;
    lastv = np;
    p = np;
    np = piece(__builtin_amdgcn_readfirstlane(knv));
    if (lane == 0) knv = atomicAdd(&ctr, 1u);
  }
  if (acc == 0x12345679u) sink[0] = acc;
}

// grid-stride dwordx4, U loads in flight per thread
template <int U, int kNt>
__global__ __launch_bounds__(256) void k_gsread(const u32x4 *__restrict__ src, size_t n, uint32_t *sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld<kNt>(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= fold(v[u]);
  }
  if (acc == 0x12345679u) sink[0] = acc;
}

struct Variant {
  std::string name;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};
}  // namespace

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8192;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  const size_t bytes = mib << 20, nrows = bytes / 1024;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("device %s, %d CUs; %zu MiB read per launch\n", prop.gcnArchName, cus, mib);
  uint8_t *a;
  uint32_t *sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&sink, 256));
  CK(hipMemset(sink, 0, 256));
  CK(hipMemset(a, 0x5A, bytes));  // non-zero data (DVFS: zeros clock higher)
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Variant> vs;
#define NP(W, P, L, NT)                                                                                    \
  vs.push_back({std::string("np read w" #W " " #P " rows/wave lds" #L) + (NT ? " nt" : " pl"), [=](hipStream_t st) {    \
                  hipLaunchKernelGGL((k_npread<W, P, L, NT>), dim3((unsigned)((nrows + W * P - 1) / (W * P))), \
                                     dim3(W * 64), 0, st, a, (uint64_t)nrows, sink);                      \
                }, {}})
#define DYN(ROWS, LG)                                                                                       \
  vs.push_back({"dyn read " #ROWS " rows/piece C=2^" #LG, [=](hipStream_t st) {                           \
                  hipLaunchKernelGGL((k_dynread<ROWS, LG>), dim3(cus), dim3(1024), 0, st, a,                \
                                     (uint64_t)(nrows / ROWS), sink);                                      \
                }, {}})
#define GS(U, NT, G)                                                                                         \
  vs.push_back({std::string("gs read U" #U) + (NT ? " nt " : " pl ") + #G "x256/CU", [=](hipStream_t st) {                  \
                  hipLaunchKernelGGL((k_gsread<U, NT>), dim3(cus * G), dim3(256), 0, st,                    \
                                     reinterpret_cast<const u32x4 *>(a), bytes / 16, sink);                 \
                }, {}})
  DYN(8, 7);
  DYN(4, 6);
  if (std::getenv("KREAD_DYN")) {  // hand-out piece size x chunk sweep
    DYN(4, 4);
    DYN(4, 5);
    DYN(8, 4);
    DYN(8, 5);
    DYN(8, 6);
    DYN(16, 3);
    DYN(16, 4);
    DYN(16, 5);
    DYN(16, 6);
    DYN(16, 7);
  }
  GS(4, 1, 8);
  GS(8, 1, 8);
  GS(4, 1, 16);
  NP(4, 4, 1, 1);
  NP(4, 4, 1, 0);
  NP(4, 8, 1, 1);
  NP(4, 16, 1, 1);
  NP(8, 8, 1, 1);
  NP(16, 4, 1, 1);
  NP(16, 8, 1, 1);
  NP(16, 4, 144, 1);
  NP(16, 8, 144, 1);
  NP(16, 16, 144, 1);
  NP(4, 4, 72, 1);
  NP(8, 8, 72, 1);
  for (auto &v : vs) v.run(s);
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
  std::printf("%-44s %10s %10s %8s %7s\n", "variant", "med GB/s", "best GB/s", "med ms", "% 8TB/s");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-44s %10.1f %10.1f %8.4f %7.1f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6, med,
                bytes / med / 1e6 / 80.0);
  }
  return 0;
}
