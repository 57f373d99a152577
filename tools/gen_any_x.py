"""Generate tools/build/k_crc_any_x.inc from the product's k_crc_any: the same
kernel (textually copied at build time, so the A/B stays the product's code)
with the 144 KiB of replicated LDS tables replaced by the LDS-free row step
(XTab, ds_bpermute) and the lane placement's per-lane columns (32 VGPRs) by the
workgroup's 8 KiB LDS copy (place_lq), so that it runs as kW-wave workgroups,
several per CU, instead of one 16-wave workgroup per CU.  Used by
tools/kany3.hip (round-3 study of the general kernel)."""
import sys

src = open(sys.argv[1]).read()
a = src.index("template <bool kSmallLanes>\n__global__ __launch_bounds__(kFastThreads) void k_crc_any(")
b = src.index("\n}\n", a) + 3
k = src[a:b]


def sub(old, new, count=1):
    global k
    assert k.count(old) == count, (old, k.count(old))
    k = k.replace(old, new)


sub("template <bool kSmallLanes>\n__global__ __launch_bounds__(kFastThreads) void k_crc_any(",
    "template <bool kSmallLanes, int kW, int kOcc = 1>\n"
    "__global__ __attribute__((amdgpu_waves_per_eu(kOcc))) __launch_bounds__(kW * 64) void k_crc_any_x(")
sub("  __shared__ __attribute__((aligned(16))) uint32_t lds[kFastLdsBytes / 4];\n",
    "  __shared__ __attribute__((aligned(16))) uint32_t lq[kLaneQWords];\n")
sub("  if (tid == 0) s_next = kFastWaves;\n", "  if (tid == 0) s_next = kW;\n")
sub("    for (uint32_t kk = wave;; kk += kFastWaves) {\n", "    for (uint32_t kk = wave;; kk += kW) {\n")
sub("""  fill_crc_tables(lds, tables, tid, kFastThreads);
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i++) col[i] = tables->lane[lane][i];
""", """  {  // the placement columns: one LDS copy per workgroup, every load before the first store
    constexpr uint32_t kQ = kLaneQWords / 4, kT = kW * 64, kPer = (kQ + kT - 1) / kT;
    const uint4 *gq = reinterpret_cast<const uint4 *>(&tables->lane_q[0][0][0]);
    uint4 t[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++)
      if (tid + k * kT < kQ) t[k] = gq[tid + k * kT];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++)
      if (tid + k * kT < kQ) reinterpret_cast<uint4 *>(lq)[tid + k * kT] = t[k];
  }
  const XTab TM = make_xtab(tables->tg, lane);
  const XTab TS = make_xtab(tables->s4, lane);
""")
a2 = k.index("  const uint32_t r4 = (lane & 31u) << 2;\n")
b2 = k.index("  // ---- small records, one per lane")
body = k[a2:b2]
assert "auto row_step" in body and "auto shift4" in body
k = k[:a2] + """  const bool msg = (flags & kFlagMessages) != 0;
  auto row_step = [&](uint32_t c, uint32_t w) -> uint32_t { return xapply(TM, c, w); };
  auto shift4 = [&](uint32_t x, uint32_t w) -> uint32_t { return xapply(TS, x, w); };

""" + k[b2:]
sub("wave_xor(matvec32(col, dd))", "wave_xor(place_lq(lq, lane, dd))")
open(sys.argv[2], "w").write("namespace hc {\nnamespace {\n" + k + "\n}  // namespace\n}  // namespace hc\n")
