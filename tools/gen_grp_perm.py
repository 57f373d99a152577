"""Generate tools/build/k_crc_grp_perm.inc from the product's k_crc_grp: the
same kernel (textually copied at build time, so the A/B stays the product's
code) with its chunk slot q permuted as q -> (q * perm) mod nchunks before the
block index is formed.  Used by tools/kgrp3.hip (round-3 large-batch study)."""
import re
import sys

src = open(sys.argv[1]).read()
# round 5: the kernel's work is the device function crc_grp_body (k_seg_combine
# calls it too); copy that and wrap it in a kernel of the old signature
a = src.index("template <bool kArrays, bool kXcd>\n__device__ __forceinline__ void crc_grp_body(")
b = src.index("\n}\n", a) + 3
k = src[a:b]
k = k.replace("void crc_grp_body(", "void crc_grp_perm_body(")
old = "unsigned long long *__restrict__ skip_slot, uint64_t skip_tag) {"
assert old in k
k = k.replace(old, "unsigned long long *__restrict__ skip_slot, uint64_t skip_tag, uint64_t perm, uint64_t nchunks) {")
old = "auto blk_of = [&](uint32_t k) -> uint64_t { return (((uint64_t)(k >> lg_chunk) * G + wg) << lg_chunk) | (k & cmask); };"
assert old in k
k = k.replace(old, """auto blk_of = [&](uint32_t k) -> uint64_t {
    uint64_t q = (uint64_t)(k >> lg_chunk) * G + wg;
    if (perm && q < nchunks) q = (q * perm) % nchunks;
    return (q << lg_chunk) | (k & cmask);
  };""")
a = src.index("template <bool kArrays, bool kXcd = false>\n__global__ __launch_bounds__(kFastThreads) void k_crc_grp(")
b = src.index("\n}\n", a) + 3
w = src[a:b]
w = w.replace("void k_crc_grp(", "void k_crc_grp_perm(")
old = "unsigned long long *__restrict__ skip_slot = nullptr,"
assert old in w
w = w.replace(old, "uint64_t perm, uint64_t nchunks, unsigned long long *__restrict__ skip_slot = nullptr,")
old = "crc_grp_body<kArrays, kXcd>("
assert old in w
w = w.replace(old, "crc_grp_perm_body<kArrays, kXcd>(")
old = "bad_bitmap, first_bad, tables, skip_slot, skip_tag);"
assert old in w
w = w.replace(old, "bad_bitmap, first_bad, tables, skip_slot, skip_tag, perm, nchunks);")
open(sys.argv[2], "w").write("namespace hc {\nnamespace {\n" + k + "\n" + w + "\n}  // namespace\n}  // namespace hc\n")
