// kbench.hip — A/B harness for streaming-kernel variants (one process,
// interleaved rounds, HIP-event time per launch; cdna_hip_programming.md
// §5.4 rule 24).  Not part of the product; build: make -C tools kbench.
//
//   ./kbench [block_bytes=8192] [nblocks=1000000] [rounds=8] [launches=5]
//
// Prints, per variant, the median and best algorithmic GB/s (bytes of the
// batch / launch time) and checks every CRC variant's output words against
// the production configuration's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "ab_hc_kernels.hip"
#include "r1_kernels.hip"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

namespace {

// Reference: the chip's read ceiling for this buffer -- grid-stride 16-B/lane
// loads at full occupancy, XOR-folded, one word stored per thread.
template <int kPol>
__global__ __launch_bounds__(256) void k_read_ref(const uint4 *p, size_t n16, uint32_t *out) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint8_t *q = reinterpret_cast<const uint8_t *>(p);
    uint4 a = hc::load_row<kPol>(q + 16 * i, 0), b = hc::load_row<kPol>(q + 16 * (i + stride), 0),
          c = hc::load_row<kPol>(q + 16 * (i + 2 * stride), 0), d = hc::load_row<kPol>(q + 16 * (i + 3 * stride), 0);
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += stride) {
    uint4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

struct Variant {
  std::string name;
  bool check;
  std::function<void(const hc::Batch &, int, hipStream_t)> run;
  std::vector<float> ms;
};

template <class Cfg>
Variant arrays_variant(const char *name, const uint64_t *doff, const uint32_t *dlen) {
  Variant v;
  v.name = name;
  v.check = !Cfg::kNull;
  v.run = [doff, dlen](const hc::Batch &b, int cus, hipStream_t s) {
    hipLaunchKernelGGL((hc::k_crc_fast<false, Cfg>), dim3(cus), dim3(Cfg::kWaves * 64), 0, s, b.base, doff,
                       dlen, b.stride, b.ulen, b.flags, b.nblocks, b.crc_out, b.bad_bitmap, b.first_bad,
                       b.tables);
  };
  return v;
}

template <class Cfg>
Variant fast_variant(const char *name, int grid_mult = 1) {
  Variant v;
  v.name = name;
  v.check = !Cfg::kNull;
  v.run = [grid_mult](const hc::Batch &b, int cus, hipStream_t s) {
    hipLaunchKernelGGL((hc::k_crc_fast<true, Cfg>), dim3(cus * grid_mult), dim3(Cfg::kWaves * 64), 0, s,
                       b.base, b.off, b.len, b.stride, b.ulen, b.flags, b.nblocks, b.crc_out,
                       b.bad_bitmap, b.first_bad, b.tables);
  };
  return v;
}


// LDS-staged streaming (the north star's "block staged in LDS"), timing-only:
// each wave streams its contiguous run of 1 KiB rows through a private ring of
// R LDS slots filled by global_load_lds_dwordx4 (LDS-DMA, no VGPR
// destination), reads each slot back with ds_read_b128 and XOR-folds it.
// The slot read is inline asm so hipcc's waitcnt pass does not see an LDS
// read aliasing the in-flight DMA (it would emit vmcnt(0) before every read);
// the counted vmcnt(R-1) is explicit.  Rows past the wave's end are clamped
// to its last row (read again, folded in: timing only).
typedef __attribute__((address_space(3))) void lds_void_t;
template <int W, int R, int AUX>
__global__ __launch_bounds__(W * 64) void k_glds_null(const uint8_t *base, uint64_t nrows, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[W * R * 1024];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * W + wave, NW = (uint64_t)gridDim.x * W;
  const uint64_t r0 = nrows * gw / NW, r1 = nrows * (gw + 1) / NW;
  uint8_t *myring = ring + wave * (R * 1024);
  uint32_t acc = 0;
  if (r0 < r1) {
#pragma unroll
    for (int u = 0; u < R; u++) {
      const uint64_t rr = r0 + u < r1 ? r0 + u : r1 - 1;
      __builtin_amdgcn_global_load_lds((const void *)(base + rr * 1024 + lane * 16),
                                       (lds_void_t *)(myring + u * 1024), 16, 0, AUX);
    }
    for (uint64_t k = r0; k < r1; k += R) {
#pragma unroll
      for (int u = 0; u < R; u++) {
        __builtin_amdgcn_s_waitcnt((R - 1) | (7 << 4) | (15 << 8));
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v;
        const uint32_t la = (uint32_t)(uintptr_t)(lds_void_t *)(myring + u * 1024) + lane * 16;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(la) : "memory");
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
        const uint64_t nr = k + u + R < r1 ? k + u + R : r1 - 1;
        __builtin_amdgcn_global_load_lds((const void *)(base + nr * 1024 + lane * 16),
                                         (lds_void_t *)(myring + u * 1024), 16, 0, AUX);
      }
    }
    __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
  }
  out[(size_t)blockIdx.x * W * 64 + threadIdx.x] = acc;
}

template <int W, int R, int AUX>
Variant glds_variant(const char *name, const uint8_t *buf, uint64_t nrows, uint32_t *scratch, int wg_per_cu) {
  Variant v;
  v.name = name;
  v.check = false;
  v.run = [=](const hc::Batch &, int cus, hipStream_t st) {
    hipLaunchKernelGGL((k_glds_null<W, R, AUX>), dim3(cus * wg_per_cu), dim3(W * 64), 0, st, buf, nrows, scratch);
  };
  return v;
}

template <int kW, bool kNullV = false>
Variant uni_variant(const char *name) {
  Variant v;
  v.name = name;
  v.check = !kNullV;
  v.run = [](const hc::Batch &b, int cus, hipStream_t s) {
    hipLaunchKernelGGL((hc::k_crc_uni<kW, kNullV>), dim3(cus), dim3(kW * 64), 0, s, b.base, b.stride, b.ulen,
                       b.flags, b.nblocks, b.crc_out, b.bad_bitmap, b.first_bad, b.tables);
  };
  return v;
}

}  // namespace

int main(int argc, char **argv) {
  const uint32_t B = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 8192;
  const uint64_t N = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1000000;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 8;
  const int launches = argc > 4 ? std::atoi(argv[4]) : 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("device %s (%s), %d CUs; batch %llu x %u B = %.3f GB\n", prop.name, prop.gcnArchName, cus,
              (unsigned long long)N, B, N * (double)B / 1e9);

  uint8_t *buf;
  uint32_t *crc, *crc_ref, *scratch;
  hc::DeviceTables *dt;
  CK(hipMalloc(&buf, N * B));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&crc_ref, N * 4));
  CK(hipMalloc(&scratch, 1 << 24));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hc::launch_fill(buf, nullptr, nullptr, B, B, N, 0x48756E64, cus * 16, s));

  uint64_t *doff;
  uint32_t *dlen;
  CK(hipMalloc(&doff, N * 8));
  CK(hipMalloc(&dlen, N * 4));
  {
    std::vector<uint64_t> ho(N);
    std::vector<uint32_t> hl(N, B);
    for (uint64_t i = 0; i < N; i++) ho[i] = i * B;
    CK(hipMemcpy(doff, ho.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, hl.data(), N * 4, hipMemcpyHostToDevice));
  }
  hc::Batch b{};
  b.base = buf;
  b.stride = B;
  b.ulen = B;
  b.nblocks = N;
  b.tables = dt;

  using namespace hc;
  std::vector<Variant> vs;
  // production first (the reference output), then the orders A/B/A/B
  vs.push_back(fast_variant<DefaultFastCfg>("w16 r4 nt (prod)"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 0>>("w16 r4 nt contiguous"));
  vs.push_back(uni_variant<16>("k_crc_uni w16"));
  vs.push_back(uni_variant<16, true>("NULL k_crc_uni w16"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 1>>("w16 r4 nt interleaved"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 0>>("w16 r4 nt contiguous (again)"));
  vs.push_back(uni_variant<16>("k_crc_uni w16 (again)"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 1>>("w16 r4 nt interleaved (again)"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 0, true>>("NULL w16 r4 nt contiguous"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 1, true>>("NULL w16 r4 nt interleaved"));
  // LDS-staged rows (LDS-DMA ring; tables leave room for 24 KiB of ring)
  vs.push_back(fast_variant<FastCfg<12, 2, 1, 0, false, true, 2>>("LDS-DMA w12 r2 nt s4x2"));
  vs.push_back(fast_variant<FastCfg<16, 2, 1, 1, false, true, 0>>("LDS-DMA w16 r2 nt s4 VALU interleaved"));
  vs.push_back(fast_variant<FastCfg<16, 2, 1, 1, true, true, 0>>("NULL LDS-DMA w16 r2 nt interleaved"));
  vs.push_back(fast_variant<FastCfg<8, 3, 1, 0, true, true, 2>>("NULL LDS-DMA w8 r3 nt"));
  const uint64_t nrows = N * B / 1024;
  vs.push_back(glds_variant<8, 3, 2>("NULL glds LDS-staged w8 r3 nt", buf, nrows, scratch, 1));
  for (int pol = 0; pol < 2; pol++) {
    Variant v;
    v.name = pol ? "REF grid-stride read nt, 8x256/CU" : "REF grid-stride read, 8x256/CU";
    v.check = false;
    v.run = [scratch, buf, N, B, pol](const hc::Batch &, int cus, hipStream_t st) {
      if (pol)
        hipLaunchKernelGGL(k_read_ref<1>, dim3(cus * 8), dim3(256), 0, st, reinterpret_cast<const uint4 *>(buf),
                           (size_t)N * B / 16, scratch);
      else
        hipLaunchKernelGGL(k_read_ref<0>, dim3(cus * 8), dim3(256), 0, st, reinterpret_cast<const uint4 *>(buf),
                           (size_t)N * B / 16, scratch);
    };
    vs.push_back(v);
  }

  // reference output
  b.crc_out = crc_ref;
  vs[0].run(b, cus, s);
  CK(hipStreamSynchronize(s));
  std::vector<uint32_t> ref(N), got(N);
  CK(hipMemcpy(ref.data(), crc_ref, N * 4, hipMemcpyDeviceToHost));
  b.crc_out = crc;

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &v : vs)  // warm + correctness
    if (v.check) {
      CK(hipMemsetAsync(crc, 0, N * 4, s));
      v.run(b, cus, s);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(got.data(), crc, N * 4, hipMemcpyDeviceToHost));
      if (got != ref) {
        std::printf("MISMATCH in variant %s\n", v.name.c_str());
        return 3;
      }
    } else {
      v.run(b, cus, s);
    }
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs)
      for (int l = 0; l < launches; l++) {
        CK(hipEventRecord(e0, s));
        v.run(b, cus, s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms);
      }
  const double bytes = (double)N * B;
  std::printf("%-40s %10s %10s %8s %8s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med ms");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-40s %10.1f %10.1f %7.2f%% %8.4f\n", v.name.c_str(), bytes / med / 1e6, bytes / best / 1e6,
                bytes / med / 1e6 / 80.0, med);
  }
  return 0;
}
