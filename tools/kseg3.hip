// kseg3.hip -- round-3 study of the packed-record dispatch's overhead
// (bench.py --workload records: k_seg_stream alone runs ~84.5 % of 8 TB/s, the
// whole dispatch ~82.5 %).  It times, over the same 2M log-uniform records
// packed at an odd address (bench.py's "records" workload), what hc_api.cpp's
// dispatch() enqueues per call and parts of it:
//   PROD      hipMallocAsync(ws) + launch_seg + hipFreeAsync (round 4: the
//             fallback for unpacked batches runs inside k_seg_combine)
//   cached    the same kernels with a workspace allocated once
//   r3j       launch_seg's kernels with round 3's first combine (22 multiplies)
//   combine   the combine kernel alone, production's and r3j's, re-run over
//             the workspace the previous variant's stream left
//   units     plan + stream + combine with 8 KiB and 4 KiB units (production:
//             16 KiB), several chunk sizes
// Each variant runs `launches` calls back to back between two events (the
// mean includes the gaps between calls, as bench.py's bracket mode); rounds
// interleave the variants.  Every variant's CRC words are compared with PROD's.
//
//   ./kseg3 [nrecords=2000000] [rounds=5] [launches=10]
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

// round 3's first unit-local combine (binary-digit tables, 22 multiplies a
// record, two workgroups per CU), for the A/B against production's
namespace hc {
namespace {
// SegTables' binary-digit tables (pw/inv), the first unit-local combine (r3j)
__device__ __forceinline__ uint32_t r3j_tmul(const uint32_t (*t)[256], uint32_t v) {
  return xor3(t[0][v & 255u], t[1][(v >> 8) & 255u], t[2][(v >> 16) & 255u]) ^ t[3][v >> 24];
}
// LDS copy of SegTables::pw[k0 .. k0+nk) at tl[0 ..) (1024 words per table)
__device__ __forceinline__ void r3j_lds_pw(uint32_t *tl, const SegTables *st, int k0, int nk) {
  const uint32_t *src = &st->pw[k0][0][0];
  for (uint32_t i = threadIdx.x; i < (uint32_t)nk * 1024u; i += blockDim.x) tl[i] = src[i];
}
__device__ __forceinline__ uint32_t r3j_lds_tmul(const uint32_t *t, uint32_t v) {
  return xor3(t[v & 255u], t[256 + ((v >> 8) & 255u)], t[512 + ((v >> 16) & 255u)]) ^ t[768 + (v >> 24)];
}

// Per record [a, b) (events j and j+1), with U_x = x's unit and re_x = x's row
// end, everything advanced to re_b:
//   shift(crc ^ ~0, re_b - b) = H(b) ^ shift(H(a) ^ shift(~0, re_a - a), re_b - re_a)
//                               ^ shift(D, re_b - U_b),  D = raw(U_a .. U_b)
// H(x) = shift(raw(U_x .. x), re_x - x) comes from k_seg_stream, and D is the
// Horner chain over the raw CRCs of the units the record spans (none when it
// starts and ends in one unit: 70 % of config 5b's records).  So no prefix over
// the whole span is needed: round 2 computed G at every unit start with three
// scan kernels (54 us at 2M records) before this one.  k_seg_plan caps records
// at kSegMaxRecord (16 MiB, 1024 units) so a lane's chain stays short.  Then
// one inverse shift by re_b - b (SegTables).  Waves work independently
// (persistent grid, two workgroups per CU, no barrier after the table fill): an
// iteration of a wave covers kSub sub-passes of 64 events (H per lane) and 63
// records (the end event's values from the next lane by a shuffle), with every
// sub-pass's loads issued before the first is used.  The tables of row shifts
// up to 63 rows and every inverse byte shift in LDS (68 KiB).
__global__ __launch_bounds__(1024) void k_seg_combine_r3j(const uint8_t *base, const uint64_t *__restrict__ offs,
                                                      const uint32_t *__restrict__ lens, uint64_t n,
                                                      const uint32_t *__restrict__ flag,
                                                      const uint32_t *__restrict__ unit_raw,
                                                      const uint32_t *__restrict__ ev_h, uint32_t *__restrict__ crc_out,
                                                      const SegTables *__restrict__ st, uint32_t *__restrict__ taken) {
  constexpr int kPwL = 6, kInv0 = kPwL * 1024, kSub = 4;
  constexpr uint32_t kUnitRows = 1u << (kSegUnitLg - 10);
  __shared__ uint32_t tl[(kPwL + kSegInv) * 1024];
  r3j_lds_pw(tl, st, 0, kPwL);
  for (uint32_t i = threadIdx.x; i < kSegInv * 1024; i += blockDim.x) tl[kInv0 + i] = (&st->inv[0][0][0])[i];
  if (taken && blockIdx.x == 0 && threadIdx.x == 0) *taken = *flag ? 0u : 1u;  // (hc_debug_seg_taken)
  __syncthreads();
  if (*flag) return;
  const SegGeo geo = seg_geo(base, offs, lens, n);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wv = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  auto rows_shift = [&](uint32_t v, uint32_t rows) {  // shift by whole rows
#pragma unroll
    for (int k = 0; k < kPwL; k++)
      if ((rows >> k) & 1u) v = r3j_lds_tmul(tl + k * 1024, v);
    rows >>= kPwL;
    for (int k = kPwL; rows; k++, rows >>= 1)
      if (rows & 1u) v = r3j_tmul(st->pw[k], v);
    return v;
  };
  for (uint64_t c = wv * 63u * kSub; c < n; c += nw * 63u * kSub) {
    uint64_t x[kSub];
    uint32_t eh[kSub];
#pragma unroll
    for (int p = 0; p < kSub; p++) {  // event c + 63p + lane (past n: the span's end again)
      const uint64_t j = c + 63u * p + lane, jj = j < n ? j : n;
      x[p] = (jj < n ? (uint64_t)base + offs[jj] : geo.pend) - geo.a0;
      eh[p] = ev_h[jj];
    }
#pragma unroll
    for (int p = 0; p < kSub; p++) {
      const uint64_t j = c + 63u * p + lane;
      const uint32_t re = (uint32_t)(x[p] >> 10) + 1u;  // the row end, in rows from A0
      const uint32_t kb = __shfl_down(eh[p], 1), rb = __shfl_down(re, 1);
      const uint64_t xb = __shfl_down((unsigned long long)x[p], 1);
      if (lane < 63 && j < n) {
        const uint32_t da = (uint32_t)(((uint64_t)re << 10) - x[p]), db = (uint32_t)(((uint64_t)rb << 10) - xb);
        // H(a) ^ shift(~0, d_a), advanced to re_b
        const uint32_t v = rows_shift(eh[p] ^ st->ones[da - 1], rb - re);
        // D = raw(U_a .. U_b): the whole units the record spans, advanced to re_b
        const uint64_t ua = x[p] >> kSegUnitLg, ub = xb >> kSegUnitLg;
        uint32_t d = 0;
        for (uint64_t u = ua; u < ub; u++) d = r3j_lds_tmul(tl + 4 * 1024, d) ^ unit_raw[u];  // 16 rows = pw[4]
        const uint32_t dd = ua < ub ? rows_shift(d, rb - (uint32_t)(ub * kUnitRows)) : 0u;
        uint32_t y = kb ^ v ^ dd;
#pragma unroll
        for (int k = 0; k < kSegInv; k++)
          if ((db >> k) & 1u) y = r3j_lds_tmul(tl + kInv0 + k * 1024, y);
        crc_out[j] = y ^ 0xFFFFFFFFu;
      }
    }
  }
}

}  // namespace
}  // namespace hc

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
}  // namespace

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 10;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  // log-uniform 64 B - 64 KiB records, back to back from byte 1
  std::mt19937_64 rng(55);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  uint64_t p = 1;
  for (uint64_t i = 0; i < n; i++) {
    len[i] = (uint32_t)(64.0 * std::exp(U(rng) * std::log(1024.0)));
    off[i] = p;
    p += len[i];
  }
  const uint64_t total = p + 64, rec_bytes = p - 1;
  std::printf("device %s, %d CUs; %llu records, %.2f GB\n", prop.gcnArchName, cus, (unsigned long long)n,
              rec_bytes / 1e9);
  uint8_t *buf;
  uint64_t *doff;
  uint32_t *dlen, *crc;
  hc::DeviceTables *dt;
  hc::SegTables *dst;
  CK(hipMalloc(&buf, total));
  CK(hipMalloc(&doff, n * 8));
  CK(hipMalloc(&dlen, n * 4));
  CK(hipMalloc(&crc, n * 4));
  CK(hipMalloc(&dt, sizeof(hc::DeviceTables)));
  CK(hipMalloc(&dst, sizeof(hc::SegTables)));
  {
    hc::DeviceTables h;
    hc::build_device_tables(h);
    CK(hipMemcpy(dt, &h, sizeof(h), hipMemcpyHostToDevice));
    auto *s = new hc::SegTables;
    hc::build_seg_tables(*s);
    CK(hipMemcpy(dst, s, sizeof(*s), hipMemcpyHostToDevice));
    delete s;
  }
  CK(hipMemcpy(doff, off.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlen, len.data(), n * 4, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hc::launch_fill(buf, nullptr, nullptr, total, (uint32_t)total, 1, 0x5B, cus * 16, s));
  CK(hipStreamSynchronize(s));

  const uint64_t mu = hc::seg_max_units((reinterpret_cast<uintptr_t>(buf) + total) -
                                        (reinterpret_cast<uintptr_t>(buf) & ~uint64_t(1023)));
  const uint64_t wsb = hc::seg_workspace_bytes(n, mu);
  uint32_t *ws_cached;
  CK(hipMalloc(&ws_cached, wsb));
  hc::Batch b{};
  b.base = buf;
  b.off = doff;
  b.len = dlen;
  b.flags = hc::kFlagMessages;
  b.nblocks = n;
  b.crc_out = crc;
  b.tables = dt;
  auto full = [&](uint32_t *ws, hipStream_t st) {
    hc::Batch bb = b;
    CK(hc::launch_seg(bb, dst, ws, mu, cus, st, nullptr));  // (round 4: the fallback runs inside k_seg_combine)
  };
  std::vector<Variant> vs;
  vs.push_back({"PROD (mallocAsync per call)", [&](hipStream_t st) {
                  uint32_t *ws;
                  CK(hipMallocAsync(reinterpret_cast<void **>(&ws), wsb, st));
                  full(ws, st);
                  CK(hipFreeAsync(ws, st));
                }, {}});
  vs.push_back({"cached workspace", [&](hipStream_t st) { full(ws_cached, st); }, {}});
  // launch_seg's kernels with round 3's first combine (the workspace layout as launch_seg's)
  uint32_t *w_flag = ws_cached, *w_plan = ws_cached + 64, *w_fev = w_plan + hc::kSegPlanMaxWgs,
           *w_raw = w_fev + mu + 1, *w_evh = w_raw + mu;
  const uint32_t plan_wgs = (uint32_t)std::min<uint64_t>((n + 256) / 256, hc::kSegPlanWgs);  // launch_seg's default cap
  auto old_combine = [&](hipStream_t st) {
    hipLaunchKernelGGL(hc::k_seg_combine_r3j, dim3(2 * cus), dim3(1024), 0, st, b.base, b.off, b.len, n, w_flag, w_raw,
                       w_evh, crc, dst, nullptr);
  };
  auto new_combine = [&](hipStream_t st) {
    hipLaunchKernelGGL(hc::k_seg_combine, dim3(cus), dim3(1024), 0, st, b.base, b.off, b.len, n, w_flag, w_raw, w_evh,
                       crc, dst, nullptr, hc::kFlagMessages, dt);
  };
  vs.push_back({"seg only, r3j combine (22 mul)", [&](hipStream_t st) {
                  hipLaunchKernelGGL(hc::k_seg_plan, dim3(plan_wgs), dim3(256), 0, st, b.base, b.off, b.len, n, mu,
                                     w_plan, w_fev);
                  hipLaunchKernelGGL(hc::k_seg_stream, dim3(cus), dim3(hc::kFastThreads), 0, st, b.base, b.off, b.len,
                                     n, 7u, w_plan, plan_wgs, w_flag, w_fev, w_raw, w_evh, dt);
                  old_combine(st);
                }, {}});
  vs.push_back({"combine alone (prod, 6 mul)", new_combine, {}});
  vs.push_back({"combine alone (r3j, 22 mul)", old_combine, {}});
  // the unit size: 8 KiB and 4 KiB units (k_crc_grp's piece sizes) against production's 16 KiB
  const uint64_t span_b = (reinterpret_cast<uintptr_t>(buf) + total) - (reinterpret_cast<uintptr_t>(buf) & ~uint64_t(1023));
  const uint64_t mu13 = (span_b >> 13) + 2, mu12 = (span_b >> 12) + 2;
  uint32_t *ws13, *ws12;
  CK(hipMalloc(&ws13, hc::seg_workspace_bytes(n, mu13)));
  CK(hipMalloc(&ws12, hc::seg_workspace_bytes(n, mu12)));
#define SEGU(KU, WS, MU, LGC)                                                                                           \
  [&, WS, MU](hipStream_t st) {                                                                                        \
    uint32_t *f_ = WS, *pb_ = WS + 64, *fe_ = pb_ + hc::kSegPlanMaxWgs, *ur_ = fe_ + (MU) + 1, *eh_ = ur_ + (MU);        \
    hipLaunchKernelGGL(hc::k_seg_plan<KU>, dim3(plan_wgs), dim3(256), 0, st, b.base, b.off, b.len, n, (uint64_t)(MU),   \
                       pb_, fe_);                                                                                      \
    hipLaunchKernelGGL(hc::k_seg_stream<KU>, dim3(cus), dim3(hc::kFastThreads), 0, st, b.base, b.off, b.len, n,          \
                       (uint32_t)(LGC), pb_, plan_wgs, f_, fe_, ur_, eh_, dt);                                          \
    hipLaunchKernelGGL(hc::k_seg_combine<KU>, dim3(cus), dim3(1024), 0, st, b.base, b.off, b.len, n, f_, ur_, eh_, crc, \
                       dst, nullptr, hc::kFlagMessages, dt);                                                           \
  }
  vs.push_back({"seg only, 8 KiB units, chunk 128", SEGU(13, ws13, mu13, 7), {}});
  vs.push_back({"seg only, 8 KiB units, chunk 256", SEGU(13, ws13, mu13, 8), {}});
  vs.push_back({"seg only, 4 KiB units, chunk 256", SEGU(12, ws12, mu12, 8), {}});
  vs.push_back({"seg only, 4 KiB units, chunk 512", SEGU(12, ws12, mu12, 9), {}});
  vs.push_back({"seg only (cached, again)", [&](hipStream_t st) { CK(hc::launch_seg(b, dst, ws_cached, mu, cus, st, nullptr)); },
                {}});

  std::vector<uint32_t> ref(n), got(n);
  vs[0].run(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), crc, n * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto &v : vs) {
    CK(hipMemsetAsync(crc, 0, n * 4, s));
    v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), crc, n * 4, hipMemcpyDeviceToHost));
    if (got != ref) {
      std::printf("MISMATCH in variant %s\n", v.name.c_str());
      bad++;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs) {
      CK(hipEventRecord(e0, s));
      for (int l = 0; l < launches; l++) v.run(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / launches);
    }
  std::printf("%-32s %10s %10s %8s %9s\n", "variant", "med GB/s", "best GB/s", "med %pk", "med us");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("%-32s %10.1f %10.1f %7.2f%% %9.1f\n", v.name.c_str(), rec_bytes / med / 1e6, rec_bytes / best / 1e6,
                rec_bytes / med / 1e6 / 80.0, med * 1e3);
  }
  return bad ? 3 : 0;
}
