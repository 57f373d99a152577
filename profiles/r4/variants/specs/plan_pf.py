# k_seg_plan: the loads of a thread's next 4 events (grid-stride) issued
# together before any is checked
SUBS = [("""  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= n && !bad; j += step) {
    const uint64_t pj = j < n ? (uint64_t)base + offs[j] : g.pend;
    uint64_t ulo = 0;
    if (j > 0) {
      const uint64_t pp = (uint64_t)base + offs[j - 1];
      if ((j < n && offs[j] != offs[j - 1] + lens[j - 1]) || pj < pp) bad = true;
      if (lens[j - 1] > kSegMaxRecord) bad = true;  // k_seg_combine's unit chain stays <= 1025 units
      ulo = ((pp - g.a0) >> kU) + 1;
    }
    if (j >= 64 && ((pj - g.a0) >> 12) == (((uint64_t)base + offs[j - 64] - g.a0) >> 12)) bad = true;
    const uint64_t uj = (pj - g.a0) >> kU;
    if (uj >= g.units || pj < g.a0) bad = true;
    if (bad) break;
    for (uint64_t u = ulo; u <= uj; u++) first_ev[u] = (uint32_t)j;
    if (j == n)
      for (uint64_t u = uj + 1; u <= g.units; u++) first_ev[u] = (uint32_t)(n + 1);
  }""", """  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  constexpr int kQ = 4;  // events a thread checks per round, their loads issued together
  for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j0 <= n && !bad; j0 += kQ * step) {
    uint64_t oj[kQ], op[kQ], o64[kQ];
    uint32_t lp[kQ];
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      const uint64_t j = j0 + q * step;
      const uint64_t jc = j < n ? j : n - 1, jp = j > 0 && j - 1 < n ? j - 1 : 0, j64 = j >= 64 && j - 64 < n ? j - 64 : 0;
      oj[q] = offs[jc];
      op[q] = offs[jp];
      lp[q] = lens[jp];
      o64[q] = offs[j64];
    }
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      const uint64_t j = j0 + q * step;
      if (j > n || bad) break;
      const uint64_t pj = j < n ? (uint64_t)base + oj[q] : g.pend;
      uint64_t ulo = 0;
      if (j > 0) {
        const uint64_t pp = (uint64_t)base + op[q];
        if ((j < n && oj[q] != op[q] + lp[q]) || pj < pp) bad = true;
        if (lp[q] > kSegMaxRecord) bad = true;  // k_seg_combine's unit chain stays <= 1025 units
        ulo = ((pp - g.a0) >> kU) + 1;
      }
      if (j >= 64 && ((pj - g.a0) >> 12) == (((uint64_t)base + o64[q] - g.a0) >> 12)) bad = true;
      const uint64_t uj = (pj - g.a0) >> kU;
      if (uj >= g.units || pj < g.a0) bad = true;
      if (bad) break;
      for (uint64_t u = ulo; u <= uj; u++) first_ev[u] = (uint32_t)j;
      if (j == n)
        for (uint64_t u = uj + 1; u <= g.units; u++) first_ev[u] = (uint32_t)(n + 1);
    }
  }""")]
