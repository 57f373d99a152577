SUBS = [("  auto events = [&](const uint4 w, uint64_t rs, uint64_t wpos, uint64_t evm) {\n",
         "  auto events = [&](const uint4 w, uint64_t rs, uint64_t wpos, uint64_t evm) {\n"
         "    for (uint64_t m = evm; m; m &= m - 1) lane0_store_u32(ev_h + wfirst + __builtin_ctzll(m), c0 ^ w.x);\n"
         "    if (evm) return;\n")]
