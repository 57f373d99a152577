// C++ mirror (include/hunddb_crc.hpp) tests, written like the reference's Go
// tests would be: known answers, edge lengths, exact error texts, in-place
// semantics, corruption detection.  `./test_hunddb_crc cpu|gpu`.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "hunddb_crc.hpp"

namespace crc = hunddb::crc;
static int failures = 0;
#define EXPECT(cond)                                                      \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      failures++;                                                         \
    }                                                                     \
  } while (0)

static std::vector<uint8_t> rnd(size_t n, uint32_t seed) {
  std::mt19937 g(seed);
  std::vector<uint8_t> v(n);
  for (auto &b : v) b = (uint8_t)g();
  return v;
}

static void cpu_tests() {
  const char *s = "123456789";
  EXPECT(crc::GetCRC(crc::ConstBytes((const uint8_t *)s, 9)) == 0xCBF43926u);
  EXPECT(crc::GetCRC(crc::ConstBytes()) == 0u);
  std::vector<uint8_t> z(4096 - 4, 0);
  EXPECT(crc::GetCRC(z) == 0x603B0489u);
  EXPECT(crc::BLOCK_SIZE == 4096 && crc::CRC_SIZE == 4);

  // AddCRCToBlockData: len < 4 untouched, returns the same slice
  std::vector<uint8_t> small = {1, 2, 3};
  auto r = crc::AddCRCToBlockData(small);
  EXPECT(r.data() == small.data() && small[0] == 1 && small[2] == 3);
  auto blk = rnd(4096, 1);
  crc::AddCRCToBlockData(blk);
  uint32_t stored;
  std::memcpy(&stored, blk.data(), 4);
  EXPECT(stored == crc::GetCRC(crc::ConstBytes(blk.data() + 4, 4092)));

  // CheckBlockIntegrity: nil / "invalid block data" / "CRC mismatch in block"
  EXPECT(crc::CheckBlockIntegrity(blk) == nullptr);
  std::vector<uint8_t> three(3);
  auto e = crc::CheckBlockIntegrity(three);
  EXPECT(e != nullptr && e.Error_() == "invalid block data");
  std::vector<uint8_t> four(4, 0);  // CRC("") == 0 -> a zero header passes
  EXPECT(crc::CheckBlockIntegrity(four) == nullptr);
  for (int bit = 0; bit < 4096 * 8; bit += 331) {
    auto c = blk;
    c[bit / 8] ^= (uint8_t)(1u << (bit % 8));
    auto err = crc::CheckBlockIntegrity(c);
    EXPECT(err && err.Error_() == "CRC mismatch in block");
  }

  // AddCRCsToData framing
  for (size_t n : {0, 1, 4091, 4092, 4093, 8184, 8185, 20000}) {
    auto src = rnd(n, (uint32_t)n);
    auto out = crc::AddCRCsToData(src);
    EXPECT(out.size() == (n + 4091) / 4092 * 4096);
    for (size_t b = 0; b < out.size() / 4096; b++) {
      crc::ConstBytes blkb(out.data() + b * 4096, 4096);
      EXPECT(crc::CheckBlockIntegrity(blkb) == nullptr);
      size_t take = std::min<size_t>(4092, n - b * 4092);
      EXPECT(std::memcmp(out.data() + b * 4096 + 4, src.data() + b * 4092, take) == 0);
    }
  }

  // FixLastBlockCRC
  std::vector<uint8_t> short_(4095);
  auto fe = crc::FixLastBlockCRC(short_);
  EXPECT(fe && fe.Error_() == "data is too short to contain a complete block");
  auto two = rnd(8192 + 100, 9);
  EXPECT(crc::FixLastBlockCRC(two) == nullptr);
  EXPECT(crc::CheckBlockIntegrity(crc::ConstBytes(two.data() + 4096, 4096)) == nullptr);

  // size helpers (float64-ceil semantics, uint64 wrap)
  EXPECT(crc::SizeAfterAddingCRCs(4092) == 4096);
  EXPECT(crc::SizeAfterAddingCRCs(4093) == 4101);
  EXPECT(crc::SizeWithoutCRCs(4096) == 4092);
  EXPECT(crc::SizeWithoutCRCs(1) == 0xFFFFFFFFFFFFFFFDull);
}

static void gpu_tests() {
  auto data = rnd(4096 * 3000, 5);
  crc::AddCRCToBlocks(data, 4096);
  int64_t fb = 0;
  EXPECT(crc::CheckBlocksIntegrity(data, 4096, &fb) == nullptr && fb == -1);
  auto words = crc::CRCBlocks(data, 4096);
  for (size_t i = 0; i < words.size(); i += 97) {
    uint32_t st;
    std::memcpy(&st, data.data() + i * 4096, 4);
    EXPECT(words[i] == st);
  }
  data[4096 * 2999 + 17] ^= 0x40;
  auto e = crc::CheckBlocksIntegrity(data, 4096, &fb);
  EXPECT(e && e.Error_() == "CRC mismatch in block" && fb == 2999);
  auto big = rnd(4092 * 700 + 5, 11);  // >= 256 blocks -> GPU framing path
  auto out = crc::AddCRCsToData(big);
  for (size_t b = 0; b < out.size() / 4096; b++)
    EXPECT(crc::CheckBlockIntegrity(crc::ConstBytes(out.data() + b * 4096, 4096)) == nullptr);
}

int main(int argc, char **argv) {
  std::string mode = argc > 1 ? argv[1] : "cpu";
  if (mode == "cpu") cpu_tests();
  if (mode == "gpu") gpu_tests();
  if (mode == "nogpu") {  // batch entries must fail loudly without a GPU
    try {
      std::vector<uint8_t> d(4096 * 4);
      crc::CRCBlocks(d, 4096);
      failures++;
    } catch (const crc::LibraryError &e) {
      EXPECT(e.code == HC_E_NODEV);
    }
  }
  std::printf("%s: %d failures\n", mode.c_str(), failures);
  return failures ? 1 : 0;
}
