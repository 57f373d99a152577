"""Generate tools/build/k_crc_grp_perm.inc from the product's k_crc_grp: the
same kernel (textually copied at build time, so the A/B stays the product's
code) with its chunk slot q permuted as q -> (q * perm) mod nchunks before the
block index is formed.  Used by tools/kgrp3.hip (round-3 large-batch study)."""
import re
import sys

src = open(sys.argv[1]).read()
a = src.index("template <bool kArrays, bool kXcd = false>\n__global__ __launch_bounds__(kFastThreads) void k_crc_grp(")
b = src.index("\n}\n", a) + 3
k = src[a:b]
k = k.replace("void k_crc_grp(", "void k_crc_grp_perm(")
old = "unsigned long long *__restrict__ skip_slot = nullptr,"
assert old in k
k = k.replace(old, "uint64_t perm, uint64_t nchunks, unsigned long long *__restrict__ skip_slot = nullptr,")
old = "auto blk_of = [&](uint32_t k) -> uint64_t { return (((uint64_t)(k >> lg_chunk) * G + wg) << lg_chunk) | (k & cmask); };"
assert old in k
k = k.replace(old, """auto blk_of = [&](uint32_t k) -> uint64_t {
    uint64_t q = (uint64_t)(k >> lg_chunk) * G + wg;
    if (perm && q < nchunks) q = (q * perm) % nchunks;
    return (q << lg_chunk) | (k & cmask);
  };""")
open(sys.argv[2], "w").write("namespace hc {\nnamespace {\n" + k + "\n}  // namespace\n}  // namespace hc\n")
