# timing only (wrong digests): k_md5's stage pieces loaded from 16-B aligned
# addresses, to see what the unaligned loads of unaligned records cost
SUBS = [
    ("        R[q] = *(gpiece)(t + (pj < e.z ? pj : e.z));",
     "        R[q] = *(gpiece)((t & ~15ull) + (pj < e.z ? pj : e.z));"),
]
