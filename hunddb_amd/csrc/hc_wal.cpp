// hc_wal.cpp — WAL recovery over a run of written WAL blocks (row f3):
// lsm/wal/wal.go:362-455 (recoverMemtable + processBlockForRecovery) with the
// per-block CheckBlockIntegrity replaced by one verify batch (hc_verify_blocks).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/hundcrc.h"
#include "hc_util.hpp"

using namespace hc;

namespace {
// One parsed piece of a WAL block (wal_header.go:5-23 framing).
struct WalItem {
  enum Kind : uint8_t { kFull, kFrag, kLast, kClear, kErrType, kErrTrunc } kind;
  uint64_t blk;
  uint32_t hdr;  // offset of the piece's header in its block (or of the error)
  uint32_t pay;  // payload offset
  uint64_t len;  // payload length
};

// processBlockForRecovery (wal.go:412-453) for one block, as items.  Returns
// false after an error item (the caller stops scanning).
bool wal_scan_block(const uint8_t *b, uint32_t bs, uint64_t blk, uint64_t off, std::vector<WalItem> &out) {
  // the rest of the block is padding iff off > last non-zero byte (:415-419)
  int64_t last = (int64_t)bs - 1;
  while (last >= 0 && b[last] == 0) last--;
  while (off < bs) {
    if ((int64_t)off > last) {
      out.push_back({WalItem::kClear, blk, (uint32_t)off, 0, 0});
      return true;
    }
    if (off + 17 > bs) {  // DeserializeWALHeader returns nil; Go then panics
      out.push_back({WalItem::kErrTrunc, blk, (uint32_t)off, 0, 0});
      return false;
    }
    uint64_t size;
    std::memcpy(&size, b + off, 8);
    const uint8_t type = b[off + 8];
    const uint32_t hdr = (uint32_t)off;
    off += 17;
    if (size > bs - off) {  // block[offset:offset+size] out of range: Go panics
      out.push_back({WalItem::kErrTrunc, blk, (uint32_t)off, 0, 0});
      return false;
    }
    WalItem::Kind k;
    if (type == 4) k = WalItem::kFull;                      // FRAGMENT_FULL
    else if (type == 1 || type == 2) k = WalItem::kFrag;    // FIRST, MIDDLE
    else if (type == 3) k = WalItem::kLast;                 // LAST
    else {
      out.push_back({WalItem::kErrType, blk, (uint32_t)(off + size), 0, 0});
      return false;
    }
    out.push_back({k, blk, hdr, (uint32_t)off, size});
    off += size;
  }
  return true;
}
}  // namespace

int hc_wal_replay(const uint8_t *blocks, uint64_t nblocks, uint32_t block_size, uint64_t start_block,
                  uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t rec_buf_cap,
                  uint64_t *rec_off, uint64_t *rec_len, uint64_t rec_slots, uint64_t *nrec, uint64_t *pos_block,
                  uint64_t *pos_offset, int64_t *bad_block) {
  if (!nrec || !pos_block || !pos_offset) return HC_E_ARG;
  if (bad_block) *bad_block = -1;
  *nrec = 0;
  *pos_block = start_block;
  *pos_offset = start_offset;
  const uint64_t bs = block_size;
  if (bs < 32 || (nblocks > start_block && !blocks) || start_offset < HC_CRC_SIZE) return HC_E_ARG;
  if (start_block >= nblocks) return HC_OK;
  const uint64_t n = nblocks - start_block;
  const uint8_t *base = blocks + start_block * bs;
  // The verify batch (wal.go:383; GPU from 256 blocks) runs on the calling
  // thread while a second thread scans, merges and copies the records out
  // without waiting for it (none of that depends on the CRCs).  The result is
  // then cut where the Go loop would have stopped: at the first bad block.
  static const uint64_t gpu_min = (uint64_t)env_int("HC_WAL_GPU_MIN_BLOCKS", 256);
  static const int threads_cfg = std::max(1, env_int("HC_WAL_THREADS", 16));  // 16: the GPU box's CPU share
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads_cfg, n / 64));
  int64_t first_bad = -1;
  int vrc = HC_OK;
  // merge outcome
  enum Stop { kAll, kErr, kFull, kCap } stop = kAll;
  uint64_t stop_blk = 0;  // block of the error / of the record that filled the memtable / of the record that did not fit
  int err_code = HC_OK;
  uint64_t pb = 0, po = HC_CRC_SIZE, count = 0;
  std::vector<uint64_t> rec_done_blk;  // block in which each record completed
  parallel_for(2, [&](int role) {
    if (role == 0) {
      if (n >= gpu_min || force_gpu()) {
        vrc = hc_verify_blocks(base, nullptr, nullptr, bs, block_size, n, nullptr, &first_bad);
      } else {
        for (uint64_t i = 0; i < n && first_bad < 0; i++)
          if (hc_check_block(base + i * bs, bs) != HC_OK) first_bad = (int64_t)i;
      }
      return;
    }
    // 1. scan the blocks into items, T threads over contiguous block ranges
    std::vector<std::vector<WalItem>> items(T);
    parallel_for(T, [&](int t) {
      const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
      items[t].reserve((hi - lo) * 2 + 4);
      for (uint64_t i = lo; i < hi; i++)
        if (!wal_scan_block(base + i * bs, block_size, start_block + i, i == 0 ? start_offset : HC_CRC_SIZE,
                            items[t]))
          break;
    });
    // 2. sequential merge: fragment reassembly, memtable-full stop, capacity stop
    struct Piece {
      const uint8_t *p;
      uint64_t len, dst;
    };
    std::vector<Piece> pieces, pending;
    uint64_t used = 0, pend_len = 0, pend_blk = 0, pend_hdr = 0;
    pb = start_block + n;
    auto emit = [&](const WalItem &it, uint64_t first_blk, uint64_t first_hdr) -> bool {
      const uint64_t len = pend_len + it.len;
      if (count >= rec_slots || used + len > rec_buf_cap || !rec_buf || !rec_off || !rec_len) {
        stop = kCap;  // resumable: the record starts at (first_blk, first_hdr)
        stop_blk = first_blk;
        pb = first_blk;
        po = first_hdr;
        return false;
      }
      rec_off[count] = used;
      rec_len[count] = len;
      for (auto &q : pending) {
        pieces.push_back({q.p, q.len, used});
        used += q.len;
      }
      pieces.push_back({base + (it.blk - start_block) * bs + it.pay, it.len, used});
      used += it.len;
      rec_done_blk.push_back(it.blk);
      count++;
      pending.clear();
      pend_len = 0;
      return true;
    };
    for (int t = 0; t < T && stop == kAll; t++) {
      for (const WalItem &it : items[t]) {
        if (it.kind == WalItem::kClear) {
          pending.clear();
          pend_len = 0;
          continue;
        }
        if (it.kind == WalItem::kErrType || it.kind == WalItem::kErrTrunc) {
          stop = kErr;
          stop_blk = it.blk;
          err_code = it.kind == WalItem::kErrType ? HC_ERR_WAL_FRAGMENT_TYPE : HC_ERR_WAL_TRUNCATED;
          pb = it.blk;
          po = it.hdr;
          break;
        }
        if (it.kind == WalItem::kFrag) {
          if (pending.empty()) {
            pend_blk = it.blk;
            pend_hdr = it.hdr;
          }
          pending.push_back({base + (it.blk - start_block) * bs + it.pay, it.len, 0});
          pend_len += it.len;
          continue;
        }
        const bool frag = it.kind == WalItem::kLast && !pending.empty();
        if (!emit(it, frag ? pend_blk : it.blk, frag ? pend_hdr : it.hdr)) break;
        if (max_records && count >= max_records) {  // memtable.IsFull: next block (wal.go:392-397)
          stop = kFull;
          stop_blk = it.blk;
          pb = it.blk + 1;
          po = HC_CRC_SIZE;
          break;
        }
      }
    }
    // 3. copy the record bytes out, T threads
    const int C = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)T, used >> 22));
    parallel_for(C, [&](int t) {
      const uint64_t lo = pieces.size() * t / C, hi = pieces.size() * (t + 1) / C;
      for (uint64_t i = lo; i < hi; i++) std::memcpy(rec_buf + pieces[i].dst, pieces[i].p, pieces[i].len);
    });
  });
  if (vrc < 0) return vrc;
  int code = stop == kErr ? err_code : HC_OK;
  if (first_bad >= 0) {
    const uint64_t B = start_block + (uint64_t)first_bad;
    // the Go loop checks a block's CRC before parsing it: a stop at or after
    // the bad block did not happen, and no record completing there exists
    if (stop == kAll || stop_blk >= B) {
      while (count > 0 && rec_done_blk[count - 1] >= B) count--;
      code = HC_ERR_CRC_MISMATCH;
      if (bad_block) *bad_block = (int64_t)B;
      pb = B;
      po = first_bad == 0 ? start_offset : HC_CRC_SIZE;
    }
  }
  *nrec = count;
  *pos_block = pb;
  *pos_offset = po;
  return code;
}

