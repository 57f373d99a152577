# diagnostic (wrong words): events' placements with the 3-shift fold but no
# mat-vec (the folded value XOR-reduced as is)
SUBS = [
("""  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    return matvec32(col, shift4(shift4(shift4(a, b_), c), d));
  };""", """  auto place = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    return matvec32(col, shift4(shift4(shift4(a, b_), c), d));
  };
  auto placeq = [&](uint32_t a, uint32_t b_, uint32_t c, uint32_t d) -> uint32_t {
    return shift4(shift4(shift4(a, b_), c), d) ^ col[lane & 31];
  };"""),
("        const uint32_t h = wave_xor(place(c0 ^ (w.x & ~keep(q, 0))", "        const uint32_t h = wave_xor(placeq(c0 ^ (w.x & ~keep(q, 0))"),
("    const uint32_t fre = wave_xor(place(c0, c1, c2, c3));  // raw(unit .. re)\n    const uint32_t e = place(w.x, w.y, w.z, w.w);",
 "    const uint32_t fre = wave_xor(placeq(c0, c1, c2, c3));  // raw(unit .. re)\n    const uint32_t e = placeq(w.x, w.y, w.z, w.w);"),
("      const uint32_t ep = place(w.x & keep(q, 0),", "      const uint32_t ep = placeq(w.x & keep(q, 0),"),
]
