SUBS = [("  auto events = [&](const uint4 w, uint64_t rs, uint64_t wpos, uint64_t evm) {\n",
         "  auto events = [&](const uint4 w, uint64_t rs, uint64_t wpos, uint64_t evm) {\n"
         "    for (uint64_t m = evm; m; m &= m - 1) hv = lane == (uint32_t)__builtin_ctzll(m) ? c0 ^ w.x : hv;\n"
         "    if (evm) return;\n")]
