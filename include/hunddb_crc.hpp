// hunddb_crc.hpp — C++ mirror of HundDB's Go package utils/crc over the C ABI
// (hundcrc.h).  Header-only.  Same names, argument meaning and error
// behaviour as /root/reference/utils/crc/crc_util.go:10-122:
//
//   Go                                   C++ (namespace hunddb::crc)
//   const BLOCK_SIZE = 1024*uint64(4)    constexpr uint64_t BLOCK_SIZE
//   const CRC_SIZE = 4                   constexpr int CRC_SIZE
//   GetCRC([]byte) uint32                uint32_t GetCRC(span)
//   AddCRCToBlockData([]byte) []byte     span AddCRCToBlockData(span)     (in place, same span)
//   AddCRCsToData([]byte) []byte         std::vector<uint8_t> AddCRCsToData(span)
//   SizeAfterAddingCRCs(uint64) uint64   uint64_t SizeAfterAddingCRCs(uint64_t)
//   SizeWithoutCRCs(uint64) uint64       uint64_t SizeWithoutCRCs(uint64_t)
//   CheckBlockIntegrity([]byte) error    Error CheckBlockIntegrity(span)
//   FixLastBlockCRC([]byte) error        Error FixLastBlockCRC(span)
//
// `Error` plays Go's `error`: default-constructed (nil) on success, otherwise
// it carries the exact errors.New text.  Library failures (no GPU for a batch
// entry, HIP errors) throw hunddb::crc::LibraryError -- the GPU path never
// falls back to the CPU.  Batched entries (the GPU hot path) are added as
// CheckBlocksIntegrity / AddCRCToBlocks / CRCBlocks.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "hundcrc.h"

namespace hunddb {
namespace crc {

constexpr uint64_t BLOCK_SIZE = 1024 * uint64_t(4);  // crc_util.go:11
constexpr int CRC_SIZE = 4;                          // crc_util.go:12

template <class T>
struct Span {  // minimal std::span stand-in (C++17)
  T *ptr = nullptr;
  size_t len = 0;
  Span() = default;
  Span(T *p, size_t n) : ptr(p), len(n) {}
  template <class C>
  Span(C &c) : ptr(c.data()), len(c.size()) {}
  T *data() const { return ptr; }
  size_t size() const { return len; }
};
using Bytes = Span<uint8_t>;
using ConstBytes = Span<const uint8_t>;

class Error {  // Go `error`: nil or a message
 public:
  Error() = default;
  explicit Error(int code) : code_(code) {}
  explicit operator bool() const { return code_ != HC_OK; }  // err != nil
  bool operator==(std::nullptr_t) const { return code_ == HC_OK; }
  bool operator!=(std::nullptr_t) const { return code_ != HC_OK; }
  std::string Error_() const { return hc_strerror(code_); }  // err.Error()
  int code() const { return code_; }

 private:
  int code_ = HC_OK;
};

struct LibraryError : std::runtime_error {
  int code;
  explicit LibraryError(int c, const char *what)
      : std::runtime_error(std::string(what) + ": " + hc_strerror(c)), code(c) {}
};

inline Error check(int rc, const char *what) {
  if (rc < 0) throw LibraryError(rc, what);
  return Error(rc);
}

// crc_util.go:15-17
inline uint32_t GetCRC(ConstBytes data) { return hc_crc32_ieee(data.data(), data.size()); }

// crc_util.go:21-33 -- stamps data[0:4] in place, returns the same span
inline Bytes AddCRCToBlockData(Bytes data) {
  check(hc_add_crc_block(data.data(), data.size()), "AddCRCToBlockData");
  return data;
}

// crc_util.go:41-64
inline std::vector<uint8_t> AddCRCsToData(ConstBytes serialized) {
  std::vector<uint8_t> out(hc_add_crcs_size(serialized.size()));
  if (out.empty()) return out;
  if (hc_add_crcs(serialized.data(), serialized.size(), out.data(), out.size()) == (size_t)-1)
    throw LibraryError(HC_E_ARG, "AddCRCsToData");
  return out;
}

// crc_util.go:69-83
inline uint64_t SizeAfterAddingCRCs(uint64_t n) { return hc_size_after_crcs(n); }
inline uint64_t SizeWithoutCRCs(uint64_t n) { return hc_size_without_crcs(n); }

// crc_util.go:88-100
inline Error CheckBlockIntegrity(ConstBytes block) {
  return check(hc_check_block(block.data(), block.size()), "CheckBlockIntegrity");
}

// crc_util.go:106-122
inline Error FixLastBlockCRC(Bytes data) {
  return check(hc_fix_last_block(data.data(), data.size()), "FixLastBlockCRC");
}

// ---- batched entries (GPU) ----------------------------------------------------

// CRC words of every blockSize-byte block (what CheckBlockIntegrity computes).
inline std::vector<uint32_t> CRCBlocks(ConstBytes data, uint32_t blockSize) {
  const uint64_t n = data.size() / blockSize;
  std::vector<uint32_t> out(n);
  check(hc_crc32_blocks(data.data(), nullptr, nullptr, blockSize, blockSize, n, out.data()), "CRCBlocks");
  return out;
}

// Batched CheckBlockIntegrity (block_manager.go:203-235 loop): first failing
// block index (-1 if none) and its error.
inline Error CheckBlocksIntegrity(ConstBytes data, uint32_t blockSize, int64_t *firstBad = nullptr) {
  int64_t fb = -1;
  Error e = check(hc_verify_blocks(data.data(), nullptr, nullptr, blockSize, blockSize,
                                   data.size() / blockSize, nullptr, &fb),
                  "CheckBlocksIntegrity");
  if (firstBad) *firstBad = fb;
  return e;
}

// Batched AddCRCToBlockData (runs of wal.go flushBlock).
inline void AddCRCToBlocks(Bytes data, uint32_t blockSize) {
  check(hc_stamp_blocks(data.data(), nullptr, nullptr, blockSize, blockSize, data.size() / blockSize),
        "AddCRCToBlocks");
}

// ---- adjacent rows ----------------------------------------------

// block_manager.go:189-242 ReadFromDisk minus the file I/O (f1): `blocks` holds
// the blocks from startOffset/blockSize on, as read.  Every touched block is
// verified in one batch.  Returns the payload and the final physical offset,
// or the error of the first failing block (its index in *badBlock).
struct ReadResult {
  std::vector<uint8_t> data;
  uint64_t finalOffset = 0;
  Error err;
};
// `verified` (optional, ceil(ReadBlocksTouched/32) words): the block cache's
// verified bits -- set bits are not hashed again; on return the blocks this
// call verified clean are set as well (hc_read_from_disk_v).
inline uint64_t ReadBlocksTouched(uint32_t blockSize, uint64_t startOffset, uint64_t size) {
  return hc_read_blocks_touched(blockSize, startOffset, size);
}
inline ReadResult ReadFromDisk(ConstBytes blocks, uint32_t blockSize, uint64_t startOffset, uint64_t size,
                               int64_t *badBlock = nullptr, std::vector<uint32_t> *verified = nullptr,
                               uint64_t *hashed = nullptr) {
  ReadResult r;
  r.data.resize(size);
  int64_t bad = -1;
  if (verified) verified->resize((ReadBlocksTouched(blockSize, startOffset, size) + 31) / 32, 0u);
  r.err = check(hc_read_from_disk_v(blocks.data(), blocks.size(), blockSize, startOffset, size,
                                    verified ? verified->data() : nullptr, r.data.data(), &r.finalOffset, &bad,
                                    hashed),
                "ReadFromDisk");
  if (badBlock) *badBlock = bad;
  if (r.err) {
    r.data.clear();
    r.finalOffset = 0;
  }
  return r;
}

// wal.go:362-455 recoverMemtable over written WAL blocks (f3): the serialized
// records (what record.Deserialize receives) of one memtable, in order, and the
// position the next memtable starts from.  maxRecords plays memtable.IsFull.
struct WalReplayResult {
  std::vector<std::vector<uint8_t>> records;
  uint64_t posBlock = 0, posOffset = CRC_SIZE;
  int64_t badBlock = -1;
  Error err;
};
inline WalReplayResult WalReplay(ConstBytes blocks, uint32_t blockSize, uint64_t startBlock = 0,
                                 uint64_t startOffset = CRC_SIZE, uint64_t maxRecords = 0) {
  WalReplayResult r;
  const uint64_t nb = blocks.size() / blockSize;
  std::vector<uint8_t> buf(nb * blockSize);
  const uint64_t slots = nb * ((blockSize - CRC_SIZE) / 17 + 1);
  std::vector<uint64_t> off(slots ? slots : 1), len(slots ? slots : 1);
  uint64_t n = 0;
  r.err = check(hc_wal_replay(blocks.data(), nb, blockSize, startBlock, startOffset, maxRecords, buf.data(),
                              buf.size(), off.data(), len.data(), slots, &n, &r.posBlock, &r.posOffset,
                              &r.badBlock),
                "WalReplay");
  r.records.reserve(n);
  for (uint64_t i = 0; i < n; i++) r.records.emplace_back(buf.begin() + off[i], buf.begin() + off[i] + len[i]);
  return r;
}

}  // namespace crc
}  // namespace hunddb
