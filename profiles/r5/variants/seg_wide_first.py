# the zeroed-gap mode ahead of the small-gap mode (no gap lines read by the combine)
SUBS = [
    ("""                        : !not_small && gsum <= 0   ? kSegGapSmall
                        : !unsorted && gsum <= 0    ? kSegGapped""",
     """                        : !unsorted && gsum <= 0    ? kSegGapped
                        : !not_small && gsum <= 0   ? kSegGapSmall"""),
]
