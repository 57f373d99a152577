// hc_cpu.cpp — host CRC-32/IEEE for the single-block drop-in calls.
//
// Dispatch rule (DESIGN.md "Boundary"): a single 4-16 KiB block costs well
// under a microsecond here and a GPU round trip costs tens of microseconds,
// so GetCRC / AddCRCToBlockData / CheckBlockIntegrity / FixLastBlockCRC on
// ONE buffer run on the host (exactly as SURVEY.md 8b prescribes).  Every
// multi-block entry point runs on the GPU and fails loudly without one.
//
// Arithmetic: Go's crc32.ChecksumIEEE (/root/reference/utils/crc/crc_util.go:16)
// - PCLMULQDQ 4-lane folding when available, slicing-by-8 otherwise.
#include <cstdint>
#include <cstring>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

#include "hc_gf2.hpp"

namespace hc {

namespace {

struct Slice8 {
  uint32_t t[8][256];
  Slice8() {
    Gf2 g;
    for (int b = 0; b < 256; b++) {
      uint32_t c = g.t[b];
      t[0][b] = c;
      for (int k = 1; k < 8; k++) {
        c = (c >> 8) ^ g.t[c & 0xFF];
        t[k][b] = c;
      }
    }
  }
};

const Slice8 &slice8() {
  static const Slice8 s;
  return s;
}

// reg: the raw (non-inverted) CRC register
uint32_t update_slice8(uint32_t reg, const uint8_t *p, size_t n) {
  const auto &T = slice8().t;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= reg;
    reg = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
          T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) reg = (reg >> 8) ^ T[0][(reg ^ *p++) & 0xFF];
  return reg;
}

#if defined(__x86_64__)
bool cpu_has_clmul() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_PCLMUL) && (c & bit_SSE4_1);
}

__attribute__((target("pclmul,sse4.1"))) inline __m128i fold(__m128i acc, __m128i k, __m128i next) {
  return _mm_xor_si128(
      _mm_xor_si128(_mm_clmulepi64_si128(acc, k, 0x00), _mm_clmulepi64_si128(acc, k, 0x11)), next);
}

// Four 128-bit accumulators folded across 64-byte strides, then reduced to
// one lane and Barrett-reduced.  Fold constants are x^(k) mod P for the
// reflected polynomial (Gopal et al., Intel 2009); n >= 64, n % 16 == 0.
__attribute__((target("pclmul,sse4.1"))) uint32_t update_clmul(uint32_t reg, const uint8_t *p,
                                                                size_t n) {
  const __m128i k_512 = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);
  const __m128i k_128 = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);
  const __m128i k_64 = _mm_set_epi64x(0, 0x163cd6124LL);
  const __m128i mu_p = _mm_set_epi64x(0x1F7011641LL, 0x1DB710641LL);
  const __m128i lo32 = _mm_set_epi32(0, 0, 0, -1);
  __m128i a[4];
  for (int i = 0; i < 4; i++) a[i] = _mm_loadu_si128(reinterpret_cast<const __m128i *>(p) + i);
  a[0] = _mm_xor_si128(a[0], _mm_cvtsi32_si128(static_cast<int>(reg)));
  size_t off = 64;
  for (; off + 64 <= n; off += 64)
    for (int i = 0; i < 4; i++)
      a[i] = fold(a[i], k_512, _mm_loadu_si128(reinterpret_cast<const __m128i *>(p + off) + i));
  __m128i x = fold(fold(fold(a[0], k_128, a[1]), k_128, a[2]), k_128, a[3]);
  for (; off + 16 <= n; off += 16)
    x = fold(x, k_128, _mm_loadu_si128(reinterpret_cast<const __m128i *>(p + off)));
  x = _mm_xor_si128(_mm_srli_si128(x, 8), _mm_clmulepi64_si128(k_128, x, 0x01));
  x = _mm_xor_si128(_mm_srli_si128(x, 4), _mm_clmulepi64_si128(_mm_and_si128(x, lo32), k_64, 0x00));
  __m128i t = _mm_clmulepi64_si128(_mm_and_si128(x, lo32), mu_p, 0x10);
  t = _mm_clmulepi64_si128(_mm_and_si128(t, lo32), mu_p, 0x00);
  return static_cast<uint32_t>(_mm_extract_epi32(_mm_xor_si128(x, t), 1));
}
#endif

}  // namespace

// ChecksumIEEE(p[0:n]) continuing from a finalised crc (Go's Update()).
uint32_t cpu_crc32_update(uint32_t crc, const uint8_t *p, size_t n) {
  uint32_t reg = ~crc;
#if defined(__x86_64__)
  static const bool clmul = cpu_has_clmul();
  if (clmul && n >= 64) {
    const size_t body = n & ~size_t(15);
    reg = update_clmul(reg, p, body);
    p += body;
    n -= body;
  }
#endif
  return ~update_slice8(reg, p, n);
}

}  // namespace hc
