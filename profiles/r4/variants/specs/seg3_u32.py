U32 = [
("constexpr uint32_t kSegUnitLg = 14;", "constexpr uint32_t kSegUnitLg = 15;"),
("""  auto rsh = [&](uint32_t v, uint32_t rows) {  // rows in [0, 16]
    return rows ? seg_lds_tmul(tl + (rows - 1u) * 1024u, v) : v;
  };""", """  auto rsh = [&](uint32_t v, uint32_t rows) {  // rows in [0, 2 kSegRs]
    if (rows > (uint32_t)kSegRs) {
      v = seg_lds_tmul(tl + (kSegRs - 1u) * 1024u, v);
      rows -= kSegRs;
    }
    return rows ? seg_lds_tmul(tl + (rows - 1u) * 1024u, v) : v;
  };"""),
("for (uint64_t u = ua + 1; u < ub; u++) v = seg_lds_tmul(tl + (kUnitRows - 1u) * 1024u, v) ^ unit_raw[u];",
 "for (uint64_t u = ua + 1; u < ub; u++) v = rsh(v, kUnitRows) ^ unit_raw[u];"),
]
SUBS = U32
