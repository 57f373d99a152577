// hc_merkle.cpp — row f4: the Merkle/MD5 integrity check of SSTable data
// (lsm/sstable/sstable.go:2287-2420 CheckIntegrity) behind the C ABI.
//
//   leaves  md5.Sum(record) per record (:2358)          hc_md5_messages / hc_dev_md5_messages (GPU)
//   tree    merkle_tree.NewMerkleTree(leaves, true)       hc_merkle_levels / hc_dev_merkle_levels
//           (merkle_tree.go:36-81), as level arrays: level 0 = the leaves, each
//           odd level followed by its zero padding node, then the parents.
//   bytes   MerkleTree.Serialize (:173-187, DFS pre-order) hc_merkle_serialize
//   check   tree.Validate(Deserialize(stored)) (:115-147, :192-226) hc_merkle_validate
//
// Host MD5 of one buffer (hc_md5) is plain C++ here: md5.Sum of one record or
// of two child hashes costs well under a microsecond on a CPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/hundcrc.h"
#include "hc_kernels.hpp"
#include "hc_util.hpp"

namespace hc {
int dev_init(int device, int *cus);  // hc_api.cpp
void set_last_launch(const hc_launch_info &info);
}

using namespace hc;

namespace {
// ---- MD5, RFC 1321 ----------------------------------------------------------
constexpr uint32_t kT[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
constexpr int kS[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};

inline uint32_t rotl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

void md5_blocks(uint32_t st[4], const uint8_t *p, size_t nblk) {
  for (size_t blk = 0; blk < nblk; blk++, p += 64) {
    uint32_t M[16];
    std::memcpy(M, p, 64);  // little-endian words (x86-64)
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    for (int i = 0; i < 64; i++) {
      const int r = i >> 4;
      uint32_t f;
      int k;
      switch (r) {
        case 0: f = (b & c) | (~b & d); k = i; break;
        case 1: f = (b & d) | (c & ~d); k = (5 * i + 1) & 15; break;
        case 2: f = b ^ c ^ d; k = (3 * i + 5) & 15; break;
        default: f = c ^ (b | ~d); k = (7 * i) & 15; break;
      }
      const uint32_t t = d;
      d = c;
      c = b;
      b = b + rotl(a + f + M[k] + kT[i], kS[4 * r + (i & 3)]);
      a = t;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
  }
}

void md5(const uint8_t *p, size_t n, uint8_t out[16]) {
  uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  const size_t full = n / 64;
  md5_blocks(st, p, full);
  uint8_t tail[128] = {0};
  const size_t r = n - full * 64;
  if (r) std::memcpy(tail, p + full * 64, r);
  tail[r] = 0x80;
  const size_t tl = r < 56 ? 64 : 128;
  const uint64_t bits = (uint64_t)n * 8;
  std::memcpy(tail + tl - 8, &bits, 8);
  md5_blocks(st, tail, tl / 64);
  std::memcpy(out, st, 16);
}

// ---- level layout -------------------------------------------------------------
// Level L occupies entries [start_L, start_L + cnt_L + pad_L); pad_L = 1 when
// the level has an odd number (> 1) of nodes.  n == 0: one entry, md5("").
struct Levels {
  std::vector<uint64_t> start, cnt;  // per level, bottom (leaves) to top (root)
  uint64_t total = 0;
  explicit Levels(uint64_t n) {
    uint64_t c = n ? n : 1, s = 0;
    for (;;) {
      start.push_back(s);
      cnt.push_back(c);
      const uint64_t padded = c > 1 ? c + (c & 1) : c;
      s += padded;
      if (c <= 1) break;
      c = padded / 2;
    }
    total = s;
  }
  int top() const { return (int)start.size() - 1; }
  // a real node at level L >= 1 has both children; padding nodes and leaves none
  bool has_children(int L, uint64_t i) const { return L > 0 && i < cnt[L]; }
  const uint8_t *at(const uint8_t *lv, int L, uint64_t i) const { return lv + 16 * (start[L] + i); }
};

void levels_cpu(uint8_t *lv, uint64_t n) {
  Levels G(n);
  if (n == 0) {
    md5(nullptr, 0, lv);
    return;
  }
  for (int L = 0; L < G.top(); L++) {
    const uint64_t c = G.cnt[L];
    uint8_t *in = lv + 16 * G.start[L];
    if (c & 1) std::memset(in + 16 * c, 0, 16);  // neutral node (merkle_tree.go:60-66)
    uint8_t *out = lv + 16 * G.start[L + 1];
    const uint64_t np = G.cnt[L + 1];
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>(16, np / 4096));
    parallel_for(T, [&](int t) {
      for (uint64_t i = np * t / T; i < np * (t + 1) / T; i++) md5(in + 32 * i, 32, out + 16 * i);
    });
  }
}
}  // namespace

extern "C" {

void hc_md5(const uint8_t *p, size_t n, uint8_t out[16]) { md5(p, n, out); }

uint64_t hc_merkle_nodes(uint64_t n) { return Levels(n).total; }

uint64_t hc_md5_workspace_bytes(uint64_t n) { return md5_workspace_bytes(n); }

int hc_dev_md5_messages(int device, const void *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                        uint32_t ulen, uint64_t n, uint8_t *out16, void *workspace, void *stream) {
  if (n == 0) return HC_OK;
  if (!base || !out16 || (reinterpret_cast<uintptr_t>(out16) & 15u)) return HC_E_ARG;
  int cus = 0;
  const int st = dev_init(device, &cus);
  if (st != HC_OK) return st;
  const int prev = [] { int d = -1; return hipGetDevice(&d) == hipSuccess ? d : -1; }();
  if (prev != device) (void)hipSetDevice(device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  void *ws = workspace;
  int rc = HC_OK;
  if (!ws && md5_workspace_bytes(n) && hipMallocAsync(&ws, md5_workspace_bytes(n), s) != hipSuccess) rc = HC_E_NOMEM;
  if (rc == HC_OK && launch_md5(static_cast<const uint8_t *>(base), off, len, stride, ulen, n,
                                static_cast<uint8_t *>(ws), out16, cus, s) != hipSuccess)
    rc = HC_E_HIP;
  set_last_launch(hc_launch_info{"k_md5", 0, n, (!off && !len) ? n * (uint64_t)ulen : 0, 0, 256, 0});
  if (!workspace && ws) (void)hipFreeAsync(ws, s);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  return rc;
}

int hc_dev_merkle_levels(int device, uint8_t *levels16, uint64_t n, void *stream) {
  if (!levels16 || (reinterpret_cast<uintptr_t>(levels16) & 15u)) return HC_E_ARG;
  int cus = 0;
  const int st = dev_init(device, &cus);
  if (st != HC_OK) return st;
  const int prev = [] { int d = -1; return hipGetDevice(&d) == hipSuccess ? d : -1; }();
  if (prev != device) (void)hipSetDevice(device);
  const int rc = launch_merkle_levels(levels16, n, static_cast<hipStream_t>(stream)) == hipSuccess ? HC_OK : HC_E_HIP;
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  return rc;
}

int hc_merkle_levels(const uint8_t *leaves16, uint64_t n, uint8_t *levels16) {
  if (!levels16 || (n && !leaves16)) return HC_E_ARG;
  if (n) std::memmove(levels16, leaves16, 16 * n);
  static const uint64_t gpu_min = (uint64_t)env_int("HC_MERKLE_GPU_MIN_LEAVES", 65536);
  if (n < gpu_min && !force_gpu()) {
    levels_cpu(levels16, n);
    return HC_OK;
  }
  // one upload of the leaves, the levels on the GPU, one download
  const int device = (int)knob(kKnobDevice);
  int cus = 0;
  int rc = dev_init(device, &cus);
  if (rc != HC_OK) return rc;
  const uint64_t total = hc_merkle_nodes(n);
  const int prev = [] { int d = -1; return hipGetDevice(&d) == hipSuccess ? d : -1; }();
  if (prev != device) (void)hipSetDevice(device);
  uint8_t *d = nullptr;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) rc = HC_E_HIP;
  if (rc == HC_OK && hipMalloc(&d, 16 * total) != hipSuccess) rc = HC_E_NOMEM;
  if (rc == HC_OK && (hipMemcpyAsync(d, levels16, 16 * n, hipMemcpyHostToDevice, s) != hipSuccess ||
                      launch_merkle_levels(d, n, s) != hipSuccess ||
                      hipMemcpyAsync(levels16, d, 16 * total, hipMemcpyDeviceToHost, s) != hipSuccess ||
                      hipStreamSynchronize(s) != hipSuccess))
    rc = HC_E_HIP;
  if (d) (void)hipFree(d);
  if (s) (void)hipStreamDestroy(s);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  return rc;
}

int hc_merkle_serialize(const uint8_t *levels16, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *nbytes) {
  if (!levels16 || !nbytes) return HC_E_ARG;
  const Levels G(n);
  *nbytes = 16 * G.total;
  if (!out) return HC_OK;  // size query
  if (cap < 16 * G.total) return HC_E_ARG;
  // DFS pre-order (parent, left subtree, right subtree) with an explicit stack
  std::vector<std::pair<int, uint64_t>> stack;
  stack.reserve(2 * (G.top() + 2));
  stack.push_back({G.top(), 0});
  uint64_t pos = 0;
  while (!stack.empty()) {
    const auto [L, i] = stack.back();
    stack.pop_back();
    std::memcpy(out + 16 * pos++, G.at(levels16, L, i), 16);
    if (G.has_children(L, i)) {
      stack.push_back({L - 1, 2 * i + 1});
      stack.push_back({L - 1, 2 * i});
    }
  }
  return HC_OK;
}

int hc_merkle_validate(const uint8_t *levels16, uint64_t n, const uint8_t *stored, uint64_t stored_len, int *valid,
                       uint8_t *mism_built16, uint8_t *mism_stored16, uint64_t *nmism) {
  if (!levels16 || !valid || !nmism || (stored_len && !stored)) return HC_E_ARG;
  *valid = 0;
  *nmism = 0;
  // Deserialize (merkle_tree.go:192-226) with nothing to read gives a nil
  // root, and Validate then panics in Go; a length that is not a multiple of
  // 16 panics in DeserializeDFS's slice expression.
  if (stored_len == 0 || stored_len % 16) return HC_E_ARG;
  const Levels G(n);
  // DeserializeDFS gives every node its left child while bytes remain, so the
  // stored tree is a left chain c_0 -> c_1 -> ... -> c_{m-1}.  DeepValidate
  // (:129-147) therefore walks the built tree's left spine a_k (level top-k,
  // index 0) against c_k: it stops at equal hashes or when a side ends,
  // records the pair when both are leaves (a_k at level 0, c_k the last), and
  // goes on only while one of the two hashes is non-zero.
  static const uint8_t kZero[16] = {0};
  const uint64_t m = stored_len / 16;
  if (std::memcmp(G.at(levels16, G.top(), 0), stored, 16) == 0) {
    *valid = 1;
    return HC_OK;
  }
  for (uint64_t k = 0; k < m && (int64_t)k <= G.top(); k++) {
    const uint8_t *a = G.at(levels16, G.top() - (int)k, 0), *c = stored + 16 * k;
    if (std::memcmp(a, c, 16) == 0) break;
    const bool a_leaf = !G.has_children(G.top() - (int)k, 0), c_leaf = k + 1 == m;
    if (a_leaf && c_leaf) {
      if (mism_built16) std::memcpy(mism_built16, a, 16);
      if (mism_stored16) std::memcpy(mism_stored16, c, 16);
      *nmism = 1;
      break;
    }
    if (std::memcmp(a, kZero, 16) == 0 && std::memcmp(c, kZero, 16) == 0) break;
  }
  return HC_OK;
}

}  // extern "C"
