// kmsg.hip — A/B harness for the general kernel k_crc_any (whole-message and
// off/len block batches; config 5b's per-record GetCRC).  Not part of the
// product; build: make -C tools kmsg.
//
//   ./kmsg [nrec=2000000] [rounds=6] [launches=5]
//
// Compares the production k_crc_any with its first (unpipelined) version,
// kept below as k_crc_any_v1, on: log-uniform 64 B - 64 KiB records packed
// back to back (config 5b), equal-size 9.8 KB records, and 4092-B blocks via
// off/len in block mode with verify.  Checks that both versions' CRC words agree.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <queue>
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

namespace hc {
namespace {
// ---- first version of k_crc_any (round 1), for A/B only ----
template <int kBatch>
__global__ __launch_bounds__(kFastThreads) void k_crc_any_v1(
    const uint8_t *base, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
    uint64_t stride, uint32_t ulen, uint32_t flags, uint64_t nblocks, int only_nonfast,
    uint32_t *__restrict__ crc_out, uint32_t *__restrict__ bad_bitmap,
    unsigned long long *__restrict__ first_bad, const DeviceTables *__restrict__ tables) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t *tg = &tables->tg[0][0];
  for (uint32_t q = tid; q < kLdsMainBytes / 16; q += kFastThreads) {
    const uint32_t a = q * 16;
    const uint32_t k = ((a >> 16) << 1) | ((a >> 7) & 1u);
    const uint32_t v = tg[k * 256 + ((a >> 8) & 255u)];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + a) = make_uint4(v, v, v, v);
  }
  const uint32_t *s4 = &tables->s4[0][0];
  for (uint32_t q = tid; q < kLdsS4Bytes / 16; q += kFastThreads) {
    const uint32_t v = s4[q];
    *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) + kLdsMainBytes + q * 16) =
        make_uint4(v, v, v, v);
  }
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
  const uint32_t w0 = tables->w0;
  __syncthreads();

  const uint32_t r4 = (lane & 31u) << 2;
  const uint32_t B0 = r4, B1 = r4 | 128u, B2 = 65536u | r4, B3 = 65536u | 128u | r4;
  const uint32_t S4base = kLdsMainBytes + ((lane & 3u) << 2);
  const bool msg = (flags & kFlagMessages) != 0;
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(c, B0, 0x0c020400u));
    const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(c, B1, 0x0c020500u));
    const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(c, B2, 0x0c020600u));
    const uint32_t t3 = lds_u32(lds, __builtin_amdgcn_perm(c, B3, 0x0c020700u));
    return xor3(xor3(t0, t1, t2), t3, w);
  };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t {
    const uint32_t t0 = lds_u32(lds, S4base + ((x & 255u) << 4));
    const uint32_t t1 = lds_u32(lds, S4base + 4096u + (((x >> 8) & 255u) << 4));
    const uint32_t t2 = lds_u32(lds, S4base + 8192u + (((x >> 16) & 255u) << 4));
    const uint32_t t3 = lds_u32(lds, S4base + 12288u + ((x >> 24) << 4));
    return xor3(xor3(t0, t1, t2), t3, w);
  };

  const uint32_t wave = uni(tid >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kFastWaves + wave;
  const uint64_t W = (uint64_t)gridDim.x * kFastWaves;
  const uint64_t b0 = uni64(nblocks * gw / W), b1 = uni64(nblocks * (gw + 1) / W);

  bool reported = false;  // wave-uniform: this wave already lowered first_bad (see k_crc_fast)
  for (uint64_t g = b0; g < b1; g += 64) {
    // metadata of blocks g .. g+63, one per lane (coalesced)
    const uint64_t j = g + lane;
    uint64_t oj = 0;
    uint32_t lj = 0;
    if (j < b1) {
      oj = offs ? offs[j] : j * stride;
      lj = lens ? lens[j] : ulen;
    }
    const bool fast = (((uintptr_t)base + oj) & 15u) == 0 && (lj & 1023u) == 0 && lj != 0;
    uint64_t todo = __ballot(j < b1 && !(only_nonfast && fast));
    while (todo) {
      const uint32_t k = (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1;
      const uint64_t blk = g + k;
      // the selected entry from lane k of the sweep (k is wave-uniform).
      // readlane returns int: cast each half to uint32_t BEFORE widening, or
      // a low word >= 2^31 sign-extends into the high word (a wild address).
      const uint32_t o_lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)oj, k);
      const uint32_t o_hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(oj >> 32), k);
      const uint64_t o = ((uint64_t)o_hi << 32) | (uint64_t)o_lo;
      const uint32_t l = (uint32_t)__builtin_amdgcn_readlane(lj, k);
      const uint8_t *blkp = base + o;
      if (!msg && l < 4) {  // "invalid block data": no CRC, always bad
        if (lane == 0) {
          if (crc_out) crc_out[blk] = 0;
          if (first_bad) {
            if (bad_bitmap) atomicOr(&bad_bitmap[blk >> 5], 1u << (blk & 31));
            if (!reported) atomicMin(first_bad, (unsigned long long)blk);
          }
        }
        reported = reported || first_bad;
        continue;
      }
      const uintptr_t P = (uintptr_t)(msg ? blkp : blkp + 4);
      const uint64_t Lp = msg ? l : l - 4;
      const uint64_t Lv = Lp + 4;
      const uint32_t rows = (uint32_t)((Lv + kRowBytes - 1) / kRowBytes);
      const uint64_t z = (uint64_t)rows * kRowBytes - Lv;
      const uintptr_t A0 = P - z - 4;
      const uint32_t m = (uint32_t)(A0 & 15u), q = m >> 2, rb = m & 3u;
      const uintptr_t Abase = A0 - m;
      uint32_t c[4] = {0, 0, 0, 0};
      {
        // rows 0 and 1 may hold the virtual prefix (z zeros + W0; z + 4 <= 1027
        // bytes): aligned chunks predicated on the payload range + funnel
        // shift + masks
        constexpr int kSlow = 2;
        const uint32_t r0 = 0;
        uint4 ch0[kSlow], ch1[kSlow];
#pragma unroll
        for (int b = 0; b < kSlow; b++) {
          ch0[b] = ch1[b] = make_uint4(0, 0, 0, 0);
          if (r0 + b < rows) {
            const uintptr_t X0 = Abase + (uintptr_t)(r0 + b) * kRowBytes + 16u * lane, X1 = X0 + 16;
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            typedef const __attribute__((address_space(1))) v4u *g16;  // global_load, not flat_load
            if (X0 + 16 > P && X0 < P + Lp) {
              const v4u t = __builtin_nontemporal_load((g16)X0);
              ch0[b] = make_uint4(t.x, t.y, t.z, t.w);
            }
            if (X1 + 16 > P && X1 < P + Lp) {
              const v4u t = __builtin_nontemporal_load((g16)X1);
              ch1[b] = make_uint4(t.x, t.y, t.z, t.w);
            }
          }
        }
#pragma unroll
        for (int b = 0; b < kSlow; b++) {
          if (r0 + b < rows) {
            const uint4 fw = funnel16(ch0[b], ch1[b], q, rb);
            uint32_t w[4] = {fw.x, fw.y, fw.z, fw.w};
            const int64_t srow = (int64_t)(r0 + b) * kRowBytes - (int64_t)z - 4;
            if (srow < 0) {  // zeros, then W0, then data
              // word k2 starts d bytes before the payload: keep its bytes
              // j >= d, and bytes ob = j - d in [-4, -1] are W0's byte ob + 4,
              // i.e. the window of Y = W0 << 32 that starts at byte 8 - d
              const uint64_t Y = (uint64_t)w0 << 32;
#pragma unroll
              for (int k2 = 0; k2 < 4; k2++) {
                const int32_t d = -((int32_t)srow + 16 * (int32_t)lane + 4 * k2);
                const uint32_t dm = d <= 0 ? 0xFFFFFFFFu : (d >= 4 ? 0u : 0xFFFFFFFFu << (8 * d));
                const uint32_t wv = (d >= 1 && d <= 8) ? (uint32_t)(Y >> (64 - 8 * d)) : 0u;
                w[k2] = (w[k2] & dm) | wv;
              }
            }
            if (r0 + b == 0) {
#pragma unroll
              for (int k2 = 0; k2 < 4; k2++) c[k2] = w[k2];
            } else {
#pragma unroll
              for (int k2 = 0; k2 < 4; k2++) c[k2] = row_step(c[k2], w[k2]);
            }
          }
        }
      }
      // rows >= 2 start inside the payload (2048 > z + 4) and the last row
      // ends at P+Lp: one unaligned 16-B load per lane per row, no funnel, no
      // masks
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      typedef u32x4 u32x4_u __attribute__((aligned(1)));
      typedef const __attribute__((address_space(1))) u32x4_u *g16u;  // global_load, not flat_load
      for (uint32_t r0 = 2; r0 < rows; r0 += kBatch) {
        u32x4 v[kBatch];
#pragma unroll
        for (int b = 0; b < kBatch; b++)  // unconditional (clamped to the last row): no branch among the loads
          v[b] = __builtin_nontemporal_load(
              (g16u)(A0 + (uintptr_t)(r0 + b < rows ? r0 + b : rows - 1) * kRowBytes + 16u * lane));
#pragma unroll
        for (int b = 0; b < kBatch; b++) {
          if (r0 + b < rows) {
            c[0] = row_step(c[0], v[b].x);
            c[1] = row_step(c[1], v[b].y);
            c[2] = row_step(c[2], v[b].z);
            c[3] = row_step(c[3], v[b].w);
          }
        }
      }
      const uint32_t dd = shift4(shift4(shift4(c[0], c[1]), c[2]), c[3]);
      const uint32_t crcv = wave_xor(matvec32(col, dd)) ^ 0xFFFFFFFFu;
      // stored word (block mode), read by every lane before lane 0 stamps it
      const uint32_t st = msg ? 0u
                              : uni((uint32_t)blkp[0] | ((uint32_t)blkp[1] << 8) | ((uint32_t)blkp[2] << 16) |
                                    ((uint32_t)blkp[3] << 24));
      const bool bad = !msg && first_bad && st != crcv;  // wave-uniform
      if (lane == 0) {
        if (crc_out) crc_out[blk] = crcv;
        if (!msg && (flags & kFlagStamp)) {
          uint8_t *wp = const_cast<uint8_t *>(blkp);
          wp[0] = (uint8_t)crcv;
          wp[1] = (uint8_t)(crcv >> 8);
          wp[2] = (uint8_t)(crcv >> 16);
          wp[3] = (uint8_t)(crcv >> 24);
        }
        if (bad) {
          if (bad_bitmap) atomicOr(&bad_bitmap[blk >> 5], 1u << (blk & 31));
          if (!reported) atomicMin(first_bad, (unsigned long long)blk);
        }
      }
      reported = reported || bad;
    }
  }
}


}  // namespace
}  // namespace hc

namespace {
uint64_t sm(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
struct Case {
  std::string name;
  uint32_t flags;
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  uint64_t bytes = 0;
};
}  // namespace

int main(int argc, char **argv) {
  const uint64_t N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<Case> cases(4);
  uint64_t seed = 0x57414C;
  cases[0].name = "config5b: log-uniform 64 B-64 KiB messages";
  cases[0].flags = hc::kFlagMessages;
  cases[1].name = "equal 9815-B messages";
  cases[1].flags = hc::kFlagMessages;
  cases[2].name = "4092-B blocks via off/len, verify";
  cases[2].flags = 0;
  cases[3].name = "config5b sizes, byte-balanced per wave";
  cases[3].flags = hc::kFlagMessages;
  uint64_t maxb = 0;
  for (int c = 0; c < 3; c++) {
    Case &k = cases[c];
    k.off.resize(N);
    k.len.resize(N);
    uint64_t o = 0;
    for (uint64_t i = 0; i < N; i++) {
      uint32_t l;
      if (c == 0) {
        const double u = (double)(sm(seed) >> 11) / 9007199254740992.0;
        l = (uint32_t)std::floor(std::exp(std::log(64.0) + u * (std::log(65536.0) - std::log(64.0))));
      } else {
        l = c == 1 ? 9815 : 4092;
      }
      k.off[i] = o;
      k.len[i] = l;
      o += l;
    }
    k.bytes = o;
    maxb = std::max(maxb, o);
  }
  {  // case 3: config 5b's sizes dealt so that every wave's contiguous run has
     // about the same bytes (greedy, largest first, into the kernel's per-wave
     // index ranges): the imbalance share of config 5b's gap
    const uint64_t W = (uint64_t)cus * hc::kFastWaves;
    std::vector<uint32_t> sz(cases[0].len);
    std::sort(sz.begin(), sz.end(), std::greater<uint32_t>());
    std::vector<uint64_t> sum(W, 0), cnt(W, 0), cap(W);
    for (uint64_t w = 0; w < W; w++) cap[w] = N * (w + 1) / W - N * w / W;
    std::vector<std::vector<uint32_t>> bins(W);
    typedef std::pair<uint64_t, uint64_t> E;
    std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
    for (uint64_t w = 0; w < W; w++) pq.push({0, w});
    for (uint32_t l : sz) {
      E e = pq.top();
      pq.pop();
      bins[e.second].push_back(l);
      if (bins[e.second].size() < cap[e.second]) pq.push({e.first + l, e.second});
    }
    Case &k = cases[3];
    uint64_t o = 0;
    for (uint64_t w = 0; w < W; w++)
      for (uint32_t l : bins[w]) {
        k.off.push_back(o);
        k.len.push_back(l);
        o += l;
      }
    k.bytes = o;
  }
  std::printf("device %s (%s), %d CUs; %llu messages per case\n", prop.name, prop.gcnArchName, cus,
              (unsigned long long)N);
  uint8_t *buf;
  uint64_t *doff;
  uint32_t *dlen, *crc, *crc1, *bm;
  unsigned long long *fb;
  hc::DeviceTables *dt;
  CK(hipMalloc(&buf, maxb + 4096));
  CK(hipMalloc(&doff, N * 8));
  CK(hipMalloc(&dlen, N * 4));
  CK(hipMalloc(&crc, N * 4));
  CK(hipMalloc(&crc1, N * 4));
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
  // fill as one big block: use 1 MiB pieces
  {
    const uint64_t piece = 1 << 20, np = (maxb + 4096 + piece - 1) / piece;
    CK(hc::launch_fill(buf, nullptr, nullptr, piece, (uint32_t)piece, (maxb + 4096) / piece, 5, cus * 16, s));
    (void)np;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &k : cases) {
    CK(hipMemcpy(doff, k.off.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, k.len.data(), N * 4, hipMemcpyHostToDevice));
    auto v1 = [&](uint32_t *out) {
      hipLaunchKernelGGL((hc::k_crc_any_v1<4>), dim3(cus), dim3(hc::kFastThreads), 0, s, buf, doff, dlen,
                         (uint64_t)0, 0u, k.flags, N, 0, out, k.flags ? nullptr : bm,
                         k.flags ? nullptr : fb, dt);
    };
    auto v2 = [&](uint32_t *out, int var) {
#define KV(V)                                                                                           \
  hipLaunchKernelGGL((hc::k_crc_any<4, V>), dim3(cus), dim3(hc::kFastThreads), 0, s, buf, doff, dlen, \
                     (uint64_t)0, 0u, k.flags, N, 0, out, k.flags ? nullptr : bm, k.flags ? nullptr : fb, dt)
      switch (var) {
        case 0: KV(0); break;
        case 1: KV(1); break;
        case 2: KV(2); break;
        default: KV(3); break;
      }
#undef KV
    };
    auto run = [&](int which, uint32_t *out) {
      if (which == 0) v1(out); else v2(out, which - 1);
    };
    const int NV = 5;  // v1, then k_crc_any<4, var> for var = 0..3
    const char *names[NV] = {"v1 (round 1)", "any oob-first", "any skip-first", "any oob-first early",
                             "any skip-first early (prod)"};
    CK(hc::launch_verify_prepare(bm, fb, N, s));
    v1(crc1);
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> a(N), b(N);
    CK(hipMemcpy(a.data(), crc1, N * 4, hipMemcpyDeviceToHost));
    std::vector<uint64_t> mism(NV, 0);
    for (int w = 1; w < NV; w++) {
      CK(hc::launch_verify_prepare(bm, fb, N, s));
      CK(hipMemset(crc, 0, N * 4));
      run(w, crc);
      CK(hipStreamSynchronize(s));
      CK(hipGetLastError());
      CK(hipMemcpy(b.data(), crc, N * 4, hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < N; i++) mism[w] += a[i] != b[i];
    }
    std::vector<std::vector<float>> t(NV);
    for (int r = 0; r < rounds; r++)
      for (int w = 0; w < NV; w++)
        for (int l = 0; l < launches; l++) {
          if (!k.flags) CK(hc::launch_verify_prepare(bm, fb, N, s));
          CK(hipEventRecord(e0, s));
          run(w, w ? crc : crc1);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          t[w].push_back(ms);
        }
    std::printf("%s: %.3f GB\n", k.name.c_str(), k.bytes / 1e9);
    for (int w = 0; w < NV; w++) {
      std::sort(t[w].begin(), t[w].end());
      const double m = t[w][t[w].size() / 2];
      std::printf("  %-18s %.4f ms %7.1f GB/s (%.1f%% of 8 TB/s)  mismatches %llu\n", names[w], m, k.bytes / m / 1e6,
                  k.bytes / m / 1e6 / 80.0, (unsigned long long)mism[w]);
    }
  }
  return 0;
}
