# k_seg_combine: every sub-pass's dependent loads (ones[da - 1] and the raw
# CRCs of the first 4 units a record spans) issued before the first sub-pass
# is computed, branch-free with clamped indices
SUBS = [("""#pragma unroll
    for (int p = 0; p < kSub; p++) {
      const uint64_t j = c + 63u * p + lane;
      const uint32_t re = (uint32_t)(x[p] >> 10) + 1u;  // the row end, in rows from A0
      const uint32_t kb = __shfl_down(eh[p], 1), rb = __shfl_down(re, 1);
      const uint64_t xb = __shfl_down((unsigned long long)x[p], 1);
      if (lane < 63 && j < n) {
        const uint32_t da = (uint32_t)(((uint64_t)re << 10) - x[p]), db = (uint32_t)(((uint64_t)rb << 10) - xb);
        const uint64_t ua = x[p] >> kU, ub = xb >> kU;
        const uint32_t X = eh[p] ^ st->ones[da - 1];
        const uint32_t ue = (uint32_t)(ua + 1) * kUnitRows;  // a's unit end, in rows
        uint32_t v = rsh(X, ua < ub ? ue - re : rb - re);
        if (ua < ub) {  // the units a .. b-1 (Horner, 16 rows a step), then U_b -> re_b
          v ^= unit_raw[ua];
          for (uint64_t u = ua + 1; u < ub; u++) v = seg_lds_tmul(tl + (kUnitRows - 1u) * 1024u, v) ^ unit_raw[u];
          v = rsh(v, rb - (uint32_t)ub * kUnitRows);
        }""", """    uint32_t re_[kSub], kb_[kSub], rb_[kSub], on_[kSub], ur_[kSub][4];
    uint64_t xb_[kSub];
#pragma unroll
    for (int p = 0; p < kSub; p++) {
      re_[p] = (uint32_t)(x[p] >> 10) + 1u;  // the row end, in rows from A0
      kb_[p] = __shfl_down(eh[p], 1);
      rb_[p] = __shfl_down(re_[p], 1);
      xb_[p] = __shfl_down((unsigned long long)x[p], 1);
      const uint32_t da = (uint32_t)(((uint64_t)re_[p] << 10) - x[p]);
      on_[p] = st->ones[(da - 1u) & 1023u];
      const uint64_t ua = x[p] >> kU, ub = xb_[p] >> kU;
#pragma unroll
      for (int k = 0; k < 4; k++) ur_[p][k] = unit_raw[ua + k < ub ? ua + k : ub];
    }
#pragma unroll
    for (int p = 0; p < kSub; p++) {
      const uint64_t j = c + 63u * p + lane;
      const uint32_t re = re_[p], kb = kb_[p], rb = rb_[p];
      const uint64_t xb = xb_[p];
      if (lane < 63 && j < n) {
        const uint32_t db = (uint32_t)(((uint64_t)rb << 10) - xb);
        const uint64_t ua = x[p] >> kU, ub = xb >> kU;
        const uint32_t X = eh[p] ^ on_[p];
        const uint32_t ue = (uint32_t)(ua + 1) * kUnitRows;  // a's unit end, in rows
        uint32_t v = rsh(X, ua < ub ? ue - re : rb - re);
        if (ua < ub) {  // the units a .. b-1 (Horner, 16 rows a step), then U_b -> re_b
          v ^= ur_[p][0];
#pragma unroll
          for (int k = 1; k < 4; k++)
            if (ua + k < ub) v = seg_lds_tmul(tl + (kUnitRows - 1u) * 1024u, v) ^ ur_[p][k];
          for (uint64_t u = ua + 4; u < ub; u++) v = seg_lds_tmul(tl + (kUnitRows - 1u) * 1024u, v) ^ unit_raw[u];
          v = rsh(v, rb - (uint32_t)ub * kUnitRows);
        }""")]
