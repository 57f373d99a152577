SUBS = []  # the source file itself is the variant
