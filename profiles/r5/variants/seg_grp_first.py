# the stream's prologue prefers the k_crc_grp fallback whenever every record is
# one of its blocks (16-B aligned 4 KiB multiples) and the batch is large
# (allow_grp), before the packed and gapped modes
SUBS = [
    ("""  const uint32_t mode = !unpacked                   ? kSegPacked
                        : !not_small && gsum <= 0   ? kSegGapSmall""",
     """  const uint32_t mode = allow_grp && csum == n      ? kSegFallbackGrp
                        : !unpacked                 ? kSegPacked
                        : !not_small && gsum <= 0   ? kSegGapSmall"""),
]
