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

#include "../hunddb_amd/csrc/hc_kernels.hip"

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
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 0>>("w16 r4 nt (prod)"));
  vs.push_back(arrays_variant<FastCfg<16, 4, 1, 0>>("w16 r4 nt, off/len arrays path", doff, dlen));
  vs.push_back(fast_variant<FastCfg<16, 3, 1, 0>>("w16 r3 nt"));
  vs.push_back(fast_variant<FastCfg<16, 5, 1, 0>>("w16 r5 nt"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 1>>("w16 r4 nt inter"));
  vs.push_back(fast_variant<FastCfg<16, 4, 4, 0>>("w16 r4 buf sc1|nt"));
  vs.push_back(fast_variant<FastCfg<12, 4, 1, 0>>("w12 r4 nt"));
  vs.push_back(fast_variant<FastCfg<16, 4, 1, 0, true>>("NULL w16 r4 nt"));
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
