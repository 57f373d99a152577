// hc_gf2.hpp — GF(2) arithmetic for CRC-32/IEEE in the reflected domain and
// the constant tables the gfx950 kernels read.
//
// Notation (used throughout DESIGN.md and the kernels):
//   raw(m)        CRC register after feeding message m into a zero register
//                 (no init, no xorout).  raw is GF(2)-linear in m and
//                 raw(a || b) = shift(raw(a), |b|) ^ raw(b).
//   shift(c, n)   register c after feeding n zero bytes = c * x^(8n) mod P.
//   ChecksumIEEE(m) = raw(W0 || m) ^ 0xFFFFFFFF with shift(W0, 4) = 0xFFFFFFFF,
//                 i.e. Go's init ^0 is a 4-byte virtual prefix W0 (any |m|).
// The reference arithmetic is Go's crc32.ChecksumIEEE as called by
// /root/reference/utils/crc/crc_util.go:16,94.
#pragma once
#include <cstdint>

namespace hc {

constexpr uint32_t kPolyReflected = 0xEDB88320u;
constexpr uint32_t kRowBytes = 1024;  // one wave-instruction of 16 B/lane
constexpr uint32_t kLanes = 64;

// Byte-at-a-time Sarwate table (host side only).
struct Gf2 {
  uint32_t t[256];
  Gf2() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int b = 0; b < 8; b++) c = (c >> 1) ^ (kPolyReflected & (0u - (c & 1u)));
      t[i] = c;
    }
  }
  uint32_t shift_bytes(uint32_t c, uint64_t n) const {
    for (uint64_t i = 0; i < n; i++) c = (c >> 8) ^ t[c & 0xFF];
    return c;
  }
  // Inverse of shift(., 4) by Gaussian elimination over GF(2).
  uint32_t unshift4(uint32_t target) const {
    uint32_t col[32];
    for (int i = 0; i < 32; i++) col[i] = shift_bytes(1u << i, 4);
    // Solve sum_i x_i col[i] = target.  Rows = output bits.
    uint64_t rows[32];  // bits 0..31: coefficient of x_i; bit 32: rhs
    for (int r = 0; r < 32; r++) {
      uint64_t v = 0;
      for (int i = 0; i < 32; i++) v |= (uint64_t)((col[i] >> r) & 1u) << i;
      v |= (uint64_t)((target >> r) & 1u) << 32;
      rows[r] = v;
    }
    int rank = 0;
    int pivcol[32];
    for (int c = 0; c < 32 && rank < 32; c++) {
      int p = -1;
      for (int r = rank; r < 32; r++)
        if ((rows[r] >> c) & 1) { p = r; break; }
      if (p < 0) continue;
      uint64_t tmp = rows[p]; rows[p] = rows[rank]; rows[rank] = tmp;
      for (int r = 0; r < 32; r++)
        if (r != rank && ((rows[r] >> c) & 1)) rows[r] ^= rows[rank];
      pivcol[rank++] = c;
    }
    uint32_t x = 0;
    for (int r = 0; r < rank; r++)
      if ((rows[r] >> 32) & 1) x |= 1u << pivcol[r];
    return x;
  }
};

// Device constant image (one per device, 32.75 KiB), uploaded once.
//   tg[k][b]   = shift(b << 8k, kRowBytes)        Horner step across a row
//   s4[k][b]   = shift(b << 8k, 4)                lane stream combine
//   lane[l][i] = shift(1 << i, kRowBytes - 12 - 16 l)   lane placement
//   w0         = shift^-1(0xFFFFFFFF, 4)           Go's init as a prefix word
//   lane_q[q][l][r] = lane[l][4q + r]              the placement columns regrouped
//                    for a workgroup-shared LDS copy read by ds_read_b128
//   sh512[0][k][b] = shift(b << 8k, 512), sh512[1][k][b] = shift^-1(b << 8k, 512)
//                    k_crc_grp's paired placement (two blocks, one mat-vec)
struct DeviceTables {
  uint32_t tg[4][256];
  uint32_t s4[4][256];
  uint32_t lane[kLanes][32];
  uint32_t w0;
  uint32_t pad[63];
  uint32_t lane_q[8][kLanes][4];
  uint32_t sh4k[4][32];  // columns of shift(., 4096 (j+1) bytes), j = 0..2 (k_unframe's group combine); [3] unused
  // k_crc_grp's paired placement: [0][k][b] = shift(b << 8k, 512), [1][k][b] = shift^-1(b << 8k, 512)
  uint32_t sh512[2][4][256];
};
static_assert(sizeof(DeviceTables) % 256 == 0, "keep the image 256-B multiple");

struct Mat32;
inline void build_sh512(DeviceTables &d);
inline void build_device_tables(DeviceTables &d) {
  Gf2 g;
  for (int k = 0; k < 4; k++)
    for (uint32_t b = 0; b < 256; b++) {
      d.tg[k][b] = g.shift_bytes(b << (8 * k), kRowBytes);
      d.s4[k][b] = g.shift_bytes(b << (8 * k), 4);
    }
  for (uint32_t l = 0; l < kLanes; l++)
    for (int i = 0; i < 32; i++) d.lane[l][i] = g.shift_bytes(1u << i, kRowBytes - 12 - 16 * l);
  d.w0 = g.unshift4(0xFFFFFFFFu);
  for (auto &p : d.pad) p = 0;
  for (int q = 0; q < 8; q++)
    for (uint32_t l = 0; l < kLanes; l++)
      for (int r = 0; r < 4; r++) d.lane_q[q][l][r] = d.lane[l][4 * q + r];
  for (int j = 0; j < 4; j++)
    for (int i = 0; i < 32; i++) d.sh4k[j][i] = j < 3 ? g.shift_bytes(1u << i, 4096ull * (j + 1)) : 0u;
  build_sh512(d);
}

// 32x32 GF(2) matrix by columns: c[i] = M e_i (host side only).
struct Mat32 {
  uint32_t c[32];
};
inline uint32_t mat_apply(const Mat32 &m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; i < 32; i++)
    if ((v >> i) & 1u) r ^= m.c[i];
  return r;
}
inline Mat32 mat_mul(const Mat32 &a, const Mat32 &b) {  // a o b
  Mat32 r;
  for (int i = 0; i < 32; i++) r.c[i] = mat_apply(a, b.c[i]);
  return r;
}
inline Mat32 mat_inverse(const Mat32 &m) {  // Gauss-Jordan on [M | I]
  uint32_t row[32], inv[32];
  for (int r = 0; r < 32; r++) {
    row[r] = 0;
    for (int i = 0; i < 32; i++) row[r] |= ((m.c[i] >> r) & 1u) << i;
    inv[r] = 1u << r;
  }
  for (int c = 0; c < 32; c++) {
    int p = c;
    while (p < 32 && !((row[p] >> c) & 1u)) p++;
    if (p == 32) continue;  // singular: never, x is invertible mod P
    uint32_t t = row[p]; row[p] = row[c]; row[c] = t;
    t = inv[p]; inv[p] = inv[c]; inv[c] = t;
    for (int r = 0; r < 32; r++)
      if (r != c && ((row[r] >> c) & 1u)) {
        row[r] ^= row[c];
        inv[r] ^= inv[c];
      }
  }
  Mat32 out;  // inv as rows -> columns
  for (int i = 0; i < 32; i++) {
    out.c[i] = 0;
    for (int r = 0; r < 32; r++) out.c[i] |= ((inv[r] >> i) & 1u) << r;
  }
  return out;
}
inline Mat32 shift_mat(const Gf2 &g, uint64_t n) {
  Mat32 m;
  for (int i = 0; i < 32; i++) m.c[i] = g.shift_bytes(1u << i, n);
  return m;
}

inline void build_sh512(DeviceTables &d) {
  Gf2 g;
  const Mat32 f = shift_mat(g, 512), inv = mat_inverse(f);
  for (int k = 0; k < 4; k++)
    for (uint32_t b = 0; b < 256; b++) {
      d.sh512[0][k][b] = mat_apply(f, b << (8 * k));
      d.sh512[1][k][b] = mat_apply(inv, b << (8 * k));
    }
}

// Constant image of the packed-record path (k_seg_*; 164 KiB, global memory):
//   pw[k][j][b]  = shift(b << 8j, 1024 * 2^k)     shift by whole rows
//   inv[k][j][b] = shift^-1(b << 8j, 2^k)          inverse shift by bytes
//   ones[d-1]    = shift(0xFFFFFFFF, d), d = 1..1024
//   rs[s-1][j][b] = shift(b << 8j, 1024 * s), s = 1..16    (k_seg_combine: one
//                   multiply per row shift inside a unit)
//   iv[..][j][b]  = shift^-1(b << 8j, e) for the octal digits of e - 1,
//                   e = 1..1024 (kSegIvD0..: 8 + 7 + 7 + 1 tables)
// pw and inv (binary digits) serve the A/B builds under tools/.
constexpr int kSegPw = 29;   // rows up to 2^29 (2^39 bytes)
constexpr int kSegInv = 11;  // byte distances 1 .. 1024
constexpr int kSegRs = 16;   // row shifts 1 .. 16 (one unit)
constexpr int kSegIvD1 = 8, kSegIvD2 = 15, kSegIvD3 = 22, kSegIv = 23;
struct SegTables {
  uint32_t pw[kSegPw][4][256];
  uint32_t inv[kSegInv][4][256];
  uint32_t ones[1024];
  uint32_t rs[kSegRs][4][256];
  uint32_t iv[kSegIv][4][256];
  uint32_t sh1[256];  // shift(v, 1): the byte-at-a-time (Sarwate) step, k_seg_combine's small gaps
};

inline void build_seg_tables(SegTables &t) {
  Gf2 g;
  auto fill = [](uint32_t (&tab)[4][256], const Mat32 &m) {
    for (int j = 0; j < 4; j++)
      for (uint32_t b = 0; b < 256; b++) tab[j][b] = mat_apply(m, b << (8 * j));
  };
  Mat32 m = shift_mat(g, kRowBytes);
  for (int k = 0; k < kSegPw; k++) {
    fill(t.pw[k], m);
    m = mat_mul(m, m);
  }
  Mat32 v = mat_inverse(shift_mat(g, 1));
  for (int k = 0; k < kSegInv; k++) {
    fill(t.inv[k], v);
    v = mat_mul(v, v);
  }
  for (int r = 1; r <= kSegRs; r++) fill(t.rs[r - 1], shift_mat(g, (uint64_t)kRowBytes * r));
  // inverse shifts: digit 0 by v + 1 bytes (v = 0..7), digit 1 by 8v, digit 2
  // by 64v (v = 1..7), digit 3 by 512
  Mat32 ip[1025];
  ip[0] = shift_mat(g, 0);
  ip[1] = mat_inverse(shift_mat(g, 1));
  for (int e = 2; e <= 1024; e++) ip[e] = mat_mul(ip[e - 1], ip[1]);
  for (int v = 0; v < 8; v++) fill(t.iv[v], ip[v + 1]);
  for (int v = 1; v < 8; v++) {
    fill(t.iv[kSegIvD1 + v - 1], ip[8 * v]);
    fill(t.iv[kSegIvD2 + v - 1], ip[64 * v]);
  }
  fill(t.iv[kSegIvD3], ip[512]);
  const Mat32 s1 = shift_mat(g, 1);
  for (uint32_t v = 0; v < 256; v++) t.sh1[v] = mat_apply(s1, v);
  uint32_t c = 0xFFFFFFFFu;
  for (int d = 1; d <= 1024; d++) {
    c = g.shift_bytes(c, 1);
    t.ones[d - 1] = c;
  }
}

}  // namespace hc
