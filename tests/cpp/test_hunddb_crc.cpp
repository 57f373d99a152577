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

  // ReadFromDisk (block_manager.go:189-242) over a 6-block image
  std::vector<uint8_t> img;
  for (int b = 0; b < 6; b++) {
    auto blkb = rnd(4096, 100 + b);
    crc::AddCRCToBlockData(blkb);
    img.insert(img.end(), blkb.begin(), blkb.end());
  }
  // `blocks` starts at block startOffset / blockSize (here block 1)
  auto rr = crc::ReadFromDisk(crc::ConstBytes(img.data() + 4096, img.size() - 4096), 4096, 4096 + 2, 3 * 4092);
  EXPECT(rr.err == nullptr && rr.data.size() == 3 * 4092);
  EXPECT(std::memcmp(rr.data.data(), img.data() + 4096 + 4, 4092) == 0);  // clamped to offset 4
  EXPECT(rr.finalOffset == crc::SizeAfterAddingCRCs(crc::SizeWithoutCRCs(4096 + 2) + 3 * 4092));
  auto badimg = img;
  badimg[3 * 4096 + 999] ^= 1;
  int64_t badb = -2;
  auto rb = crc::ReadFromDisk(badimg, 4096, 0, 5 * 4092, &badb);
  EXPECT(rb.err && rb.err.Error_() == "CRC mismatch in block" && badb == 3 && rb.data.empty());
  // the block cache's verified bits: block 3 masked (a verified cached copy) is
  // trusted and not hashed; the other 4 are, and come back marked
  std::vector<uint32_t> vbits(1, 1u << 3);
  uint64_t hashed = 0;
  auto rv = crc::ReadFromDisk(badimg, 4096, 0, 5 * 4092, &badb, &vbits, &hashed);
  EXPECT(rv.err == nullptr && hashed == 4 && vbits[0] == 0x1Fu && crc::ReadBlocksTouched(4096, 0, 5 * 4092) == 5);

  // WalReplay (wal.go:362-455): one FULL record + a 2-fragment record
  std::vector<uint8_t> wal(3 * 4096, 0);
  auto put_hdr = [&](size_t at, uint64_t size, uint8_t type) {
    std::memcpy(&wal[at], &size, 8);
    wal[at + 8] = type;
    uint64_t log = 1;
    std::memcpy(&wal[at + 9], &log, 8);
  };
  auto rec1 = rnd(100, 7);
  put_hdr(4, rec1.size(), 4);
  std::memcpy(&wal[4 + 17], rec1.data(), rec1.size());
  auto rec2 = rnd(4075 + 500, 8);
  put_hdr(4096 + 4, 4075, 1);
  std::memcpy(&wal[4096 + 21], rec2.data(), 4075);
  put_hdr(2 * 4096 + 4, 500, 3);
  std::memcpy(&wal[2 * 4096 + 21], rec2.data() + 4075, 500);
  for (int b = 0; b < 3; b++) crc::AddCRCToBlockData(crc::Bytes(wal.data() + b * 4096, 4096));
  auto wr = crc::WalReplay(wal, 4096);
  EXPECT(wr.err == nullptr && wr.records.size() == 2 && wr.records[0] == rec1 && wr.records[1] == rec2);
  EXPECT(wr.posBlock == 3 && wr.posOffset == 4);
  auto w1 = crc::WalReplay(wal, 4096, 0, 4, 1);  // memtable full after one record: next block
  EXPECT(w1.err == nullptr && w1.records.size() == 1 && w1.posBlock == 1);
  wal[2 * 4096 + 300] ^= 2;
  auto wb = crc::WalReplay(wal, 4096);
  EXPECT(wb.err && wb.err.Error_() == "CRC mismatch in block" && wb.badBlock == 2 && wb.records.size() == 1);

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
