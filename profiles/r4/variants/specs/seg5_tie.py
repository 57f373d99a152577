# the row as one 128-bit asm operand where it is folded: the loop-carried
# row then stays in its load's register tuple (no copies at the loop latch)
TIE = [("""  auto row = [&](uint4 &q, uint64_t rs, uint64_t wpos, __amdgpu_buffer_rsrc_t rn, uint32_t no) {
    const uint4 w = q;
""", """  auto row = [&](uint4 &q, uint64_t rs, uint64_t wpos, __amdgpu_buffer_rsrc_t rn, uint32_t no) {
    typedef unsigned int r32x4 __attribute__((ext_vector_type(4)));
    r32x4 qq = __builtin_bit_cast(r32x4, q);
    asm volatile("" : "+v"(qq));
    const uint4 w = __builtin_bit_cast(uint4, qq);
""")]
SUBS = TIE
