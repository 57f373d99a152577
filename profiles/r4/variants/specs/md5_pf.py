# k_md5: the next block's 16 message words read from LDS before the current
# block is compressed (branch-free block loop: lanes past their stage's blocks
# are masked off; the wave skips a block no lane has)
SUBS = [("""    for (uint32_t b = 0; b < (uint32_t)kStage; b++) {
      if (b < t.nb) {
        uint32_t M[16];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          const u32x4 v = L[lane * kPitch + 4u * b + q];
          M[4 * q] = v.x;
          M[4 * q + 1] = v.y;
          M[4 * q + 2] = v.z;
          M[4 * q + 3] = v.w;
        }
        md5_compress(st, M);
      }
    }""", """    u32x4 mv[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) mv[q] = L[lane * kPitch + q];
#pragma unroll
    for (uint32_t b = 0; b < (uint32_t)kStage; b++) {
      uint32_t M[16];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        M[4 * q] = mv[q].x;
        M[4 * q + 1] = mv[q].y;
        M[4 * q + 2] = mv[q].z;
        M[4 * q + 3] = mv[q].w;
      }
      if (b + 1 < (uint32_t)kStage) {
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) mv[q] = L[lane * kPitch + 4u * (b + 1) + q];
      }
      if (!__ballot(b < t.nb)) break;
      uint32_t s2[4] = {st[0], st[1], st[2], st[3]};
      md5_compress(s2, M);
      if (b < t.nb) {
        st[0] = s2[0];
        st[1] = s2[1];
        st[2] = s2[2];
        st[3] = s2[3];
      }
    }""")]
