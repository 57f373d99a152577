SUBS = []
