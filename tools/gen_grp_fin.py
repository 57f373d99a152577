"""Generate tools/build/k_crc_grp_fin.inc from the product's k_crc_grp: the
same kernel (textually copied at build time) with a kFin template switch on
the per-block finalise, for tools/kgrp4.hip (what the finalise costs at 4 KiB):
  kFin 0  the product's finalise (a copy: words checked)
  kFin 1  timing-only: crc = wave XOR of c0 ^ c1 ^ c2 ^ c3 (no shift4, no placement)
  kFin 2  timing-only: the three shift4 kept, the lane placement mat-vec dropped"""
import sys

src = open(sys.argv[1]).read()
a = src.index("template <bool kArrays, bool kXcd = false>\n__global__ __launch_bounds__(kFastThreads) void k_crc_grp(")
b = src.index("\n}\n", a) + 3
k = src[a:b]
k = k.replace("template <bool kArrays, bool kXcd = false>", "template <bool kArrays, bool kXcd, int kFin>")
k = k.replace("void k_crc_grp(", "void k_crc_grp_fin(")
old = """        const uint32_t d = shift4(shift4(shift4(c0, c1), c2), c3);
        const uint32_t crc = wave_xor(matvec32(col, d)) ^ 0xFFFFFFFFu;"""
assert old in k
k = k.replace(old, """        uint32_t crc;
        if constexpr (kFin == 1) {
          crc = wave_xor(c0 ^ c1 ^ c2 ^ c3);
        } else if constexpr (kFin == 2) {
          crc = wave_xor(shift4(shift4(shift4(c0, c1), c2), c3));
        } else {
          const uint32_t d = shift4(shift4(shift4(c0, c1), c2), c3);
          crc = wave_xor(matvec32(col, d)) ^ 0xFFFFFFFFu;
        }""")
open(sys.argv[2], "w").write("namespace hc {\nnamespace {\n" + k + "\n}  // namespace\n}  // namespace hc\n")
