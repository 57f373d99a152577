// kmd5.hip — A/B harness for the MD5 leaf kernel (row f4).  Not part of the
// product; build: make -C tools kmd5.
//
//   ./kmd5 [nrec=2000000] [rounds=5] [launches=3]
//
// Over the same records (log-uniform 64 B - 64 KiB packed back to back at an
// odd address, and 4096-B records at 4096-B stride):
//   v1          the first kernel (kept below): lane per message, each lane
//               loading its own 64-B blocks; tail slots by k_md5_v1_tail
//   v1 loads    v1's memory pattern, XOR fold instead of the compression
//   v1 alu      v1's control flow and compression, no data loads
//   prod        launch_md5: k_md5 (staged through LDS, tails padded in LDS)
//   prod main   k_md5 alone
// plus memory-pattern probes (4096-B records, XOR fold): each lane reading its
// own record in 64..512-B chunks, and a wave reading 64 records in rotation
// with 64..1024-B contiguous pieces per record per instruction.
// Digests of prod are compared with v1's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../hunddb_amd/csrc/hc_md5.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

namespace hc {
namespace {

// ---------------------------------------------------------------------------
// Thread per message: the 128-byte tail slot = the message's last len % 64 data
// bytes, 0x80, zeros and the 64-bit little-endian bit length at byte 56 (tail
// < 56 bytes: one block) or 120 (two blocks).  The data bytes come from the
// aligned dwords that hold them (an aligned dword holding a message byte never
// leaves that byte's page), shifted per lane with v_alignbyte.
__global__ __launch_bounds__(256) void k_md5_v1_tail(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
                                                  const uint32_t *__restrict__ lens, uint64_t stride, uint32_t ulen,
                                                  uint64_t n, uint8_t *__restrict__ tails) {
  for (uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = offs ? offs[m] : m * stride;
    const uint32_t l = lens ? lens[m] : ulen;
    const uint32_t r = l & 63u;
    const uintptr_t tp = (uintptr_t)base + o + (l & ~63u);
    const uint32_t sh = (uint32_t)(tp & 3u);
    const uint32_t *A = reinterpret_cast<const uint32_t *>(tp - sh);
    const uint32_t nd = r ? (sh + r + 3) >> 2 : 0u;  // aligned dwords holding the tail bytes (<= 17)
    uint32_t dw[17];
#pragma unroll
    for (int j = 0; j < 17; j++) dw[j] = (uint32_t)j < nd ? __builtin_nontemporal_load(A + j) : 0u;
    uint32_t w[32];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t v = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], sh);
      const int32_t nb = (int32_t)r - 4 * i;  // tail bytes in this word
      v &= nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
      v |= (uint32_t)i == (r >> 2) ? (0x80u << (8 * (r & 3u))) : 0u;
      w[i] = v;
    }
#pragma unroll
    for (int i = 16; i < 32; i++) w[i] = 0;
    const uint64_t bits = (uint64_t)l * 8;
    const bool two = r >= 56;
    w[14] = two ? w[14] : (uint32_t)bits;
    w[15] = two ? w[15] : (uint32_t)(bits >> 32);
    w[30] = two ? (uint32_t)bits : 0u;
    w[31] = two ? (uint32_t)(bits >> 32) : 0u;
    uint4 *dst = reinterpret_cast<uint4 *>(tails + m * 128);
#pragma unroll
    for (int q = 0; q < 8; q++) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
}

// ---------------------------------------------------------------------------
// Lane per message, messages pulled from the wave's pool as lanes free up.
__global__ __launch_bounds__(256) void k_md5_v1(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
                                             const uint32_t *__restrict__ lens, uint64_t stride, uint32_t ulen,
                                             uint64_t n, const uint8_t *__restrict__ tails,
                                             uint8_t *__restrict__ out16) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t wave = uni_u32(threadIdx.x >> 6);
  const uint64_t wpb = blockDim.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + wave, W = (uint64_t)gridDim.x * wpb;
  const uint64_t p1 = n * (gw + 1) / W;
  uint64_t next = n * gw / W;  // wave-uniform pool cursor
  bool act = false;
  uint64_t msg = 0;
  const uint8_t *p = nullptr;   // next full data block
  const uint8_t *tp = nullptr;  // next tail block
  uint32_t nfull = 0, ntail = 0;
  uint32_t st[4] = {0, 0, 0, 0};
  for (;;) {
    const uint64_t need = __ballot(!act);
    if (need) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      const uint64_t idx = next + rank;
      next += (uint64_t)__builtin_popcountll(need);
      if (!act && idx < p1) {
        const uint64_t o = offs ? offs[idx] : idx * stride;
        const uint32_t l = lens ? lens[idx] : ulen;
        msg = idx;
        p = base + o;
        nfull = l >> 6;
        ntail = (l & 63u) < 56 ? 1u : 2u;
        tp = tails + idx * 128;
        md5_init(st);
        act = true;
      }
    }
    if (!__ballot(act)) break;
    if (act) {
      const uint8_t *src = nfull ? p : tp;
      uint32_t M[16];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(src + 16 * q));
        M[4 * q] = v.x;
        M[4 * q + 1] = v.y;
        M[4 * q + 2] = v.z;
        M[4 * q + 3] = v.w;
      }
      md5_compress(st, M);
      if (nfull) {
        p += 64;
        nfull--;
      } else {
        tp += 64;
        if (--ntail == 0) {
          *reinterpret_cast<uint4 *>(out16 + msg * 16) = make_uint4(st[0], st[1], st[2], st[3]);
          act = false;
        }
      }
    }
  }

}

// kMode 1: loads only (XOR fold); kMode 2: compression only (no loads)
template <int kMode>
__global__ __launch_bounds__(256) void k_md5_diag(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
                                                  const uint32_t *__restrict__ lens, uint64_t stride, uint32_t ulen,
                                                  uint64_t n, const uint8_t *__restrict__ tails,
                                                  uint8_t *__restrict__ out16) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const uint32_t wave = uni_u32(threadIdx.x >> 6);
  const uint64_t wpb = blockDim.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + wave, W = (uint64_t)gridDim.x * wpb;
  const uint64_t p1 = n * (gw + 1) / W;
  uint64_t next = n * gw / W;
  bool act = false;
  uint64_t msg = 0;
  const uint8_t *p = nullptr, *tp = nullptr;
  uint32_t nfull = 0, ntail = 0;
  uint32_t st[4] = {0, 0, 0, 0};
  for (;;) {
    const uint64_t need = __ballot(!act);
    if (need) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      const uint64_t idx = next + rank;
      next += (uint64_t)__builtin_popcountll(need);
      if (!act && idx < p1) {
        const uint64_t o = offs ? offs[idx] : idx * stride;
        const uint32_t l = lens ? lens[idx] : ulen;
        msg = idx;
        p = base + o;
        nfull = l >> 6;
        ntail = (l & 63u) < 56 ? 1u : 2u;
        tp = tails + idx * 128;
        md5_init(st);
        act = true;
      }
    }
    if (!__ballot(act)) break;
    if (act) {
      const uint8_t *src = nfull ? p : tp;
      uint32_t M[16];
      if (kMode == 2) {
#pragma unroll
        for (int q = 0; q < 16; q++) M[q] = (uint32_t)(uintptr_t)src + q;
        md5_compress(st, M);
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(src + 16 * q));
          M[4 * q] = v.x;
          M[4 * q + 1] = v.y;
          M[4 * q + 2] = v.z;
          M[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int q = 0; q < 16; q++) st[q & 3] ^= M[q];
      }
      if (nfull) {
        p += 64;
        nfull--;
      } else {
        tp += 64;
        if (--ntail == 0) {
          *reinterpret_cast<uint4 *>(out16 + msg * 16) = make_uint4(st[0], st[1], st[2], st[3]);
          act = false;
        }
      }
    }
  }
}

// ---- memory-pattern probes (4096-B records at 4096-B stride, XOR fold) ----
// kCh bytes per lane per iteration from the lane's own record; kPf: the next
// iteration's loads issued before the current chunk is folded.
template <int kCh, bool kPf>
__global__ __launch_bounds__(256) void k_pat_lane(const uint8_t *__restrict__ base, uint64_t n,
                                                  uint8_t *__restrict__ out16) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kL = kCh / 16;
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, T = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = gt; r < n; r += T) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(base + r * 4096);
    u32x4 acc = {0, 0, 0, 0};
    u32x4 A[kL], B[kL];
#pragma unroll
    for (int j = 0; j < kL; j++) A[j] = __builtin_nontemporal_load(p + j);
    for (int c = 1; c <= 4096 / kCh; c++) {
      if (kPf && c < 4096 / kCh) {
#pragma unroll
        for (int j = 0; j < kL; j++) B[j] = __builtin_nontemporal_load(p + c * kL + j);
      }
#pragma unroll
      for (int j = 0; j < kL; j++) acc ^= A[j];
      if (c < 4096 / kCh) {
        if (kPf) {
#pragma unroll
          for (int j = 0; j < kL; j++) A[j] = B[j];
        } else {
#pragma unroll
          for (int j = 0; j < kL; j++) A[j] = __builtin_nontemporal_load(p + c * kL + j);
        }
      }
    }
    *reinterpret_cast<u32x4 *>(out16 + r * 16) = acc;
  }
}

// the streaming pattern: a wave reads one record with 4 x 1 KiB coalesced loads
__global__ __launch_bounds__(256) void k_pat_wave(const uint8_t *__restrict__ base, uint64_t n,
                                                  uint8_t *__restrict__ out16) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), W = (uint64_t)gridDim.x * 4;
  for (uint64_t r = gw; r < n; r += W) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(base + r * 4096);
    u32x4 acc = __builtin_nontemporal_load(p + lane);
#pragma unroll
    for (int j = 1; j < 4; j++) acc ^= __builtin_nontemporal_load(p + 64 * j + lane);
    if (lane == 0) *reinterpret_cast<u32x4 *>(out16 + r * 16) = acc;
  }
}

// pieces: a wave keeps 64 records in rotation; one visit reads kP bytes of each
// (one instruction = 1024/kP records x kP contiguous bytes), 8 instructions in
// flight, XOR fold.  The access pattern of a lane-per-message hash whose
// blocks are staged by coalesced loads.
template <int kP>
__global__ __launch_bounds__(256) void k_pat_piece(const uint8_t *__restrict__ base, uint64_t n,
                                                   uint8_t *__restrict__ out16) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kPerInst = 1024 / kP, kInst = 64 / kPerInst, kLanesPerRec = kP / 16;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), W = (uint64_t)gridDim.x * 4;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t r0 = gw * 64; r0 < n; r0 += W * 64) {
    for (int v = 0; v < 4096 / kP; v++) {
      for (int i = 0; i < kInst; i += 8) {
        u32x4 R[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const uint64_t rec = r0 + (uint64_t)(i + j) * kPerInst + lane / kLanesPerRec;
          const uint64_t a = (rec < n ? rec : 0) * 4096 + (uint64_t)v * kP + 16u * (lane % kLanesPerRec);
          R[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + a));
        }
#pragma unroll
        for (int j = 0; j < 8; j++) acc ^= R[j];
      }
    }
  }
  *reinterpret_cast<u32x4 *>(out16 + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16 % (n * 16)) = acc;
}
}  // namespace
}  // namespace hc

static uint64_t sm(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill_rand(uint32_t *p, uint64_t nw) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 12345;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

struct Case {
  std::string name;
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  uint64_t bytes = 0;
};

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 3;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<Case> cases(2);
  uint64_t seed = 0x4D4435, maxb = 0;
  cases[0].name = "log-uniform 64 B - 64 KiB records, odd start";
  cases[1].name = "4096-B records, 4096-B stride";
  for (int c = 0; c < 2; c++) {
    Case &k = cases[c];
    uint64_t o = c == 0 ? 3 : 0;
    for (uint64_t i = 0; i < N; i++) {
      uint32_t l = 4096;
      if (c == 0) {
        const double u = (double)(sm(seed) >> 11) / 9007199254740992.0;
        l = (uint32_t)std::floor(std::exp(std::log(64.0) + u * (std::log(65536.0) - std::log(64.0))));
      }
      k.off.push_back(o);
      k.len.push_back(l);
      k.bytes += l;
      o += l;
    }
    maxb = std::max(maxb, o);
  }
  std::printf("device %s (%s), %d CUs; %llu records per case\n", prop.name, prop.gcnArchName, cus,
              (unsigned long long)N);
  uint8_t *buf, *tails, *out, *ref;
  uint64_t *doff;
  uint32_t *dlen;
  CK(hipMalloc(&buf, maxb + 4096));
  CK(hipMalloc(&tails, N * 128));
  CK(hipMalloc(&out, N * 16));
  CK(hipMalloc(&ref, N * 16));
  CK(hipMalloc(&doff, N * 8));
  CK(hipMalloc(&dlen, N * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipLaunchKernelGGL(k_fill_rand, dim3(cus * 8), dim3(256), 0, s, reinterpret_cast<uint32_t *>(buf),
                     (maxb + 4096) / 4);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int NV = 8;
  const char *names[NV] = {"v1", "v1 loads", "v1 alu", "prod", "prod main", "bpermute", "S4 d1",
                           "v1 alu 2w/SIMD"};
  uint8_t *ws;
  CK(hipMalloc(&ws, hc::md5_workspace_bytes(N) + 16));
  for (auto &k : cases) {
    CK(hipMemcpy(doff, k.off.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, k.len.data(), N * 4, hipMemcpyHostToDevice));
    const uint64_t waves = std::min<uint64_t>((N + 63) / 64, (uint64_t)cus * 32);
    const int grid = (int)((waves + 3) / 4);
    hipLaunchKernelGGL(hc::k_md5_v1_tail, dim3(cus * 8), dim3(256), 0, s, buf, doff, dlen, (uint64_t)0, 0u, N, tails);
    // k_md5's grid as launch_md5 sets it
    const uint64_t pgrid = std::min<uint64_t>((N + 1023) / 1024, (uint64_t)cus * 2);
    auto run = [&](int v, uint8_t *o) {
      switch (v) {
        case 0:
          hipLaunchKernelGGL(hc::k_md5_v1, dim3(grid), dim3(256), 0, s, buf, doff, dlen, (uint64_t)0, 0u, N, tails,
                             o);
          break;
        case 1:
          hipLaunchKernelGGL(hc::k_md5_diag<1>, dim3(grid), dim3(256), 0, s, buf, doff, dlen, (uint64_t)0, 0u, N,
                             tails, o);
          break;
        case 2:
          hipLaunchKernelGGL(hc::k_md5_diag<2>, dim3(grid), dim3(256), 0, s, buf, doff, dlen, (uint64_t)0, 0u, N,
                             tails, o);
          break;
        case 3: CK(hc::launch_md5(buf, doff, dlen, 0, 0, N, ws, o, cus, s)); break;
        case 4:  // the main kernel alone, on the tail slots k_md5_v1_tail wrote (same format)
          hipLaunchKernelGGL((hc::k_md5<true, true>), dim3((unsigned)pgrid), dim3(256), 0, s, buf, doff, dlen,
                             (uint64_t)0, 0u, N, o);
          break;
#define KV(S, D, G)                                                                                              \
  hipLaunchKernelGGL((hc::k_md5<true, true, S, D>), dim3((unsigned)std::min<uint64_t>((N + 1023) / 1024, cus * G)), \
                     dim3(256), 0, s, buf, doff, dlen, (uint64_t)0, 0u, N, o)
        case 5:
          hipLaunchKernelGGL((hc::k_md5<true, true, 4, 1, false>), dim3((unsigned)pgrid), dim3(256), 0, s, buf, doff,
                             dlen, (uint64_t)0, 0u, N, o);
          break;
        case 6: KV(4, 1, 2); break;
        default:
          hipLaunchKernelGGL(hc::k_md5_diag<2>, dim3(cus * 2), dim3(256), 0, s, buf, doff, dlen, (uint64_t)0, 0u, N,
                             tails, o);
          break;
#undef KV
      }
    };
    run(0, ref);
    CK(hipStreamSynchronize(s));
    CK(hipGetLastError());
    std::vector<uint8_t> a(N * 16), b(N * 16);
    CK(hipMemcpy(a.data(), ref, N * 16, hipMemcpyDeviceToHost));
    std::vector<uint64_t> mism(NV, 0);
    for (int v = 3; v < 7; v++) {
      CK(hipMemset(out, 0, N * 16));
      run(v, out);
      CK(hipStreamSynchronize(s));
      CK(hipGetLastError());
      CK(hipMemcpy(b.data(), out, N * 16, hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < N; i++) mism[v] += std::memcmp(&a[16 * i], &b[16 * i], 16) != 0;
    }
    std::vector<std::vector<float>> t(NV);
    for (int r = 0; r < rounds; r++)
      for (int v = 0; v < NV; v++)
        for (int l = 0; l < launches; l++) {
          CK(hipEventRecord(e0, s));
          run(v, v ? out : ref);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          t[v].push_back(ms);
        }
    std::printf("%s: %.3f GB\n", k.name.c_str(), k.bytes / 1e9);
    for (int v = 0; v < NV; v++) {
      std::sort(t[v].begin(), t[v].end());
      const double m = t[v][t[v].size() / 2];
      std::printf("  %-16s %.4f ms %7.1f GB/s  mismatches %llu\n", names[v], m, k.bytes / m / 1e6,
                  (unsigned long long)mism[v]);
    }
    std::fflush(stdout);
  }
  {  // memory-pattern probes on the 4096-B case
    const uint64_t bytes = N * 4096;
    const char *pn[14] = {"lane 64B", "lane 64B pf", "lane 128B", "lane 128B pf", "lane 256B", "lane 512B",
                          "wave coalesced", "wave coalesced 2x", "piece 64", "piece 128", "piece 256", "piece 512",
                          "piece 1024", "piece 256 8w/CU"};
    for (int v = 0; v < 14; v++) {
      std::vector<float> t;
      for (int r = 0; r < rounds * launches + 1; r++) {
        CK(hipEventRecord(e0, s));
        const int g = cus * 8;
        switch (v) {
          case 0: hipLaunchKernelGGL((hc::k_pat_lane<64, false>), dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 1: hipLaunchKernelGGL((hc::k_pat_lane<64, true>), dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 2: hipLaunchKernelGGL((hc::k_pat_lane<128, false>), dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 3: hipLaunchKernelGGL((hc::k_pat_lane<128, true>), dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 4: hipLaunchKernelGGL((hc::k_pat_lane<256, false>), dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 5: hipLaunchKernelGGL((hc::k_pat_lane<512, false>), dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 6: hipLaunchKernelGGL(hc::k_pat_wave, dim3(g), dim3(256), 0, s, buf, N, out); break;
          case 7: hipLaunchKernelGGL(hc::k_pat_wave, dim3(g * 2), dim3(256), 0, s, buf, N, out); break;
          case 8: hipLaunchKernelGGL((hc::k_pat_piece<64>), dim3(cus * 4), dim3(256), 0, s, buf, N, out); break;
          case 9: hipLaunchKernelGGL((hc::k_pat_piece<128>), dim3(cus * 4), dim3(256), 0, s, buf, N, out); break;
          case 10: hipLaunchKernelGGL((hc::k_pat_piece<256>), dim3(cus * 4), dim3(256), 0, s, buf, N, out); break;
          case 11: hipLaunchKernelGGL((hc::k_pat_piece<512>), dim3(cus * 4), dim3(256), 0, s, buf, N, out); break;
          case 12: hipLaunchKernelGGL((hc::k_pat_piece<1024>), dim3(cus * 4), dim3(256), 0, s, buf, N, out); break;
          default: hipLaunchKernelGGL((hc::k_pat_piece<256>), dim3(cus * 2), dim3(256), 0, s, buf, N, out); break;
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      const double m = t[t.size() / 2];
      std::printf("  probe %-16s %.4f ms %7.1f GB/s\n", pn[v], m, bytes / m / 1e6);
    }
  }
  return 0;
}
