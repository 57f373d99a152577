// hc_wal.cpp — WAL recovery over a run of written WAL blocks (row f3):
// lsm/wal/wal.go:362-455 (recoverMemtable + processBlockForRecovery) with the
// per-block CheckBlockIntegrity replaced by one verify batch (hc_verify_blocks).
//
// Everything but a short sequential pass runs in parallel over contiguous
// block ranges (a block always starts with a header, so ranges scan
// independently):
//   A. per range (T threads): scan the blocks and merge their pieces into
//      records locally.  Only the range's "head" depends on the fragments
//      still pending from earlier ranges: the FIRST/MIDDLE pieces before the
//      range's first reset point (a LAST, which consumes the pending
//      fragments, or a padding tail, which clears them -- wal.go:415-419).
//   B. sequential over ranges: carry the pending fragments through the heads,
//      number the records and apply the stops (framing error, memtable full,
//      output capacity) -- O(ranges), plus one walk over the records of the
//      range where a stop falls.
//   C. per range (T threads): write rec_off/rec_len and copy the bytes out.
// The verify batch runs on the calling thread meanwhile (GPU from 1024 blocks,
// HC_WAL_GPU_MIN_BLOCKS);
// the result is cut where the Go loop would have stopped: at the first bad block.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include <emmintrin.h>

#include "../../include/hundcrc.h"
#include "hc_util.hpp"

using namespace hc;

namespace {
struct Piece {
  const uint8_t *p;
  uint64_t len;
};

// Fragments waiting for their LAST (Go's fragmentBuffer), as piece references.
struct Pending {
  std::vector<Piece> pieces;
  uint64_t len = 0;
  uint64_t blk = 0;  // header position of the first pending piece
  uint32_t hdr = 0;
  void add(const Piece &q, uint64_t b, uint32_t h) {
    if (pieces.empty()) {
      blk = b;
      hdr = h;
    }
    pieces.push_back(q);
    len += q.len;
  }
  void clear() {
    pieces.clear();
    len = 0;
  }
};

struct Rec {
  uint64_t piece0;     // first piece in Range::pieces
  uint32_t npieces;
  bool head;           // the head LAST: the pending fragments of earlier ranges go first
  uint64_t len;        // bytes (a head record: without that incoming prefix until phase B)
  uint64_t start_blk;  // where the record starts (resume position when it does not fit)
  uint32_t start_hdr;
  uint64_t done_blk;   // block in which it completes
};

struct Range {
  std::vector<Piece> pieces;
  std::vector<Rec> recs;
  bool reset = false;  // the range has a LAST or a padding tail
  Pending head;        // FIRST/MIDDLE pieces before the first reset
  Pending tail;        // pieces after the last reset (pending at the range end)
  int64_t head_rec = -1;
  bool err = false;
  int err_code = HC_OK;
  uint64_t err_blk = 0, err_hdr = 0;
  uint64_t bytes = 0;  // sum of local record lengths
  // phase B
  std::vector<Piece> prefix;  // incoming pending pieces of the head record
  uint64_t keep = 0;          // records kept
  uint64_t rec_base = 0, byte_base = 0;
};

// processBlockForRecovery (wal.go:412-453) for one block, feeding the range's
// local merge.  Returns false after a framing error (the range stops there).
bool scan_block(Range &R, const uint8_t *b, uint32_t bs, uint64_t blk, uint64_t off) {
  // the rest of the block is padding iff off > its last non-zero byte (:415-419)
  int64_t last = (int64_t)bs - 1;
  while (last >= 0 && b[last] == 0) last--;
  while (off < bs) {
    if ((int64_t)off > last) {  // fragmentBuffer = fragmentBuffer[:0]
      if (R.reset)
        R.tail.clear();
      R.reset = true;  // the head ends here (cleared: the incoming pending dies)
      return true;
    }
    if (off + 17 > bs) {  // DeserializeWALHeader returns nil; Go then panics
      R.err = true;
      R.err_code = HC_ERR_WAL_TRUNCATED;
      R.err_blk = blk;
      R.err_hdr = off;
      return false;
    }
    uint64_t size;
    std::memcpy(&size, b + off, 8);
    const uint8_t type = b[off + 8];
    const uint32_t hdr = (uint32_t)off;
    off += 17;
    if (size > bs - off) {  // block[offset:offset+size] out of range: Go panics
      R.err = true;
      R.err_code = HC_ERR_WAL_TRUNCATED;
      R.err_blk = blk;
      R.err_hdr = off;
      return false;
    }
    const Piece q{b + off, size};
    if (type == 4) {  // FRAGMENT_FULL: Put(payload); the fragment buffer is untouched
      R.recs.push_back({R.pieces.size(), 1, false, size, blk, hdr, blk});
      R.pieces.push_back(q);
      R.bytes += size;
    } else if (type == 1 || type == 2) {  // FIRST, MIDDLE: append
      (R.reset ? R.tail : R.head).add(q, blk, hdr);
    } else if (type == 3) {  // LAST: record = fragment buffer + payload, buffer cleared
      Pending &pd = R.reset ? R.tail : R.head;
      Rec r{R.pieces.size(), (uint32_t)pd.pieces.size() + 1, !R.reset, pd.len + size,
            pd.pieces.empty() ? blk : pd.blk, pd.pieces.empty() ? hdr : pd.hdr, blk};
      R.pieces.insert(R.pieces.end(), pd.pieces.begin(), pd.pieces.end());
      R.pieces.push_back(q);
      if (!R.reset) R.head_rec = (int64_t)R.recs.size();
      R.recs.push_back(r);
      R.bytes += r.len;
      if (R.reset) R.tail.clear();
      R.reset = true;  // (head pieces stay in R.head for phase B's start position)
    } else {
      R.err = true;
      R.err_code = HC_ERR_WAL_FRAGMENT_TYPE;
      R.err_blk = blk;
      R.err_hdr = off + size;
      return false;
    }
    off += size;
  }
  return true;
}

// Record bytes are written once and not read back here: hc::copy_nt's
// non-temporal stores skip the write-allocate read of every destination line,
// which would otherwise compete for host memory bandwidth with the verify
// batch's DMA of the same image.
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int hc_wal_replay(const uint8_t *blocks, uint64_t nblocks, uint32_t block_size, uint64_t start_block,
                  uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t rec_buf_cap,
                  uint64_t *rec_off, uint64_t *rec_len, uint64_t rec_slots, uint64_t *nrec, uint64_t *pos_block,
                  uint64_t *pos_offset, int64_t *bad_block) {
  return hc_wal_replay_v(blocks, nblocks, block_size, start_block, start_offset, max_records, rec_buf, rec_buf_cap,
                         rec_off, rec_len, nullptr, rec_slots, nrec, pos_block, pos_offset, bad_block, nullptr);
}

int hc_wal_replay_v(const uint8_t *blocks, uint64_t nblocks, uint32_t block_size, uint64_t start_block,
                    uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t rec_buf_cap,
                    uint64_t *rec_off, uint64_t *rec_len, uint64_t *rec_end_block, uint64_t rec_slots,
                    uint64_t *nrec, uint64_t *pos_block, uint64_t *pos_offset, int64_t *bad_block,
                    uint64_t *pend_pos) {
  if (pend_pos) pend_pos[0] = UINT64_MAX, pend_pos[1] = 0;
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
  const uint64_t gpu_min = (uint64_t)knob(kKnobWalGpuMin);  // hc_debug_set: tools/crossover.py
  static const int threads_cfg = std::max(1, env_int("HC_WAL_THREADS", 16));  // 16: the GPU box's CPU share
  static const int trace = env_int("HC_WAL_TRACE", 0);
  // blocks per range at least HC_WAL_MIN_RANGE (64; read per call so tests can
  // force many small ranges and exercise the cross-range merge)
  const uint64_t min_range = (uint64_t)std::max<int64_t>(1, knob(kKnobWalMinRange));
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads_cfg, n / min_range));
  const bool have_out = rec_buf && rec_off && rec_len;
  int64_t first_bad = -1;
  int vrc = HC_OK;
  enum Stop { kAll, kErr, kFull, kCap } stop = kAll;
  uint64_t stop_blk = 0;  // block of the error / of the record that filled the memtable / that did not fit
  int err_code = HC_OK;
  uint64_t pb = start_block + n, po = HC_CRC_SIZE, count = 0;
  uint64_t pend_blk = UINT64_MAX, pend_hdr = 0;  // fragments still pending when the blocks run out
  std::vector<Range> R(T);
  int last_range = T - 1;  // ranges after a stop are not used
  double t0 = now_s(), tv = 0, ta = 0, tb = 0, tc = 0;
  auto work = [&](int role) {
    if (role == 0) {
      bool on_gpu = false;
      if (n >= gpu_min || force_gpu()) {
        const int inj = injected_failure(kInjectWalReplay);
        vrc = inj ? inj : hc_verify_blocks(base, nullptr, nullptr, bs, block_size, n, nullptr, &first_bad);
        if (vrc >= 0) {  // HC_OK or the first bad block's reason
          on_gpu = true;
          vrc = HC_OK;
          g_stats.wal_gpu.fetch_add(1, std::memory_order_relaxed);
        } else if (!force_gpu() && gpu_batch_failure(vrc)) {
          // recovery fails only on a bad block or a framing error (wal.go:362-455):
          // a GPU batch that cannot run finishes on the host path
          if (vrc == HC_E_NODEV) {
            g_stats.nodev_host.fetch_add(1, std::memory_order_relaxed);
          } else {
            g_stats.wal_gpu_fallback.fetch_add(1, std::memory_order_relaxed);
            g_stats.last_fallback_error.store(vrc, std::memory_order_relaxed);
          }
          vrc = HC_OK;
          first_bad = -1;
        } else {
          on_gpu = true;  // HC_FORCE_GPU, or a caller / library error: returned
        }
      }
      if (!on_gpu)
        for (uint64_t i = 0; i < n && first_bad < 0; i++)
          if (hc_check_block(base + i * bs, bs) != HC_OK) first_bad = (int64_t)i;
      tv = now_s() - t0;
      return;
    }
    // A. scan + local merge per range
    parallel_for(T, [&](int t) {
      const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
      R[t].pieces.reserve((hi - lo) * 2 + 4);
      R[t].recs.reserve((hi - lo) + 4);
      for (uint64_t i = lo; i < hi; i++)
        if (!scan_block(R[t], base + i * bs, block_size, start_block + i, i == 0 ? start_offset : HC_CRC_SIZE))
          break;
    });
    ta = now_s() - t0;
    // B. pending fragments through the heads, numbering, stops
    Pending pend;
    uint64_t used = 0;
    for (int t = 0; t < T && stop == kAll; t++) {
      Range &G = R[t];
      last_range = t;
      if (G.head_rec >= 0) {  // the head LAST takes the incoming fragments first
        Rec &h = G.recs[(size_t)G.head_rec];
        G.prefix = pend.pieces;
        h.len += pend.len;
        G.bytes += pend.len;
        if (!pend.pieces.empty()) {
          h.start_blk = pend.blk;
          h.start_hdr = pend.hdr;
        }
      }
      if (G.reset) {
        pend = G.tail;
      } else {
        for (size_t i = 0; i < G.head.pieces.size(); i++)
          pend.add(G.head.pieces[i], G.head.blk, G.head.hdr);
      }
      G.rec_base = count;
      G.byte_base = used;
      const uint64_t nr = G.recs.size();
      const bool fits_all = have_out && count + nr <= rec_slots && used + G.bytes <= rec_buf_cap;
      const bool fills = max_records && count + nr >= max_records;
      if (fits_all && !fills) {
        G.keep = nr;
        count += nr;
        used += G.bytes;
      } else {  // a stop falls in this range: walk its records
        G.keep = 0;
        for (const Rec &r : G.recs) {
          if (!have_out || count >= rec_slots || used + r.len > rec_buf_cap) {
            stop = kCap;  // resumable: the record starts at (start_blk, start_hdr)
            stop_blk = r.start_blk;
            pb = r.start_blk;
            po = r.start_hdr;
            break;
          }
          G.keep++;
          count++;
          used += r.len;
          if (max_records && count >= max_records) {  // memtable.IsFull: next block (wal.go:392-397)
            stop = kFull;
            stop_blk = r.done_blk;
            pb = r.done_blk + 1;
            po = HC_CRC_SIZE;
            break;
          }
        }
      }
      if (stop == kAll && G.err) {
        stop = kErr;
        stop_blk = G.err_blk;
        err_code = G.err_code;
        pb = G.err_blk;
        po = G.err_hdr;
      }
    }
    if (stop == kAll && !pend.pieces.empty()) {
      pend_blk = pend.blk;
      pend_hdr = pend.hdr;
    }
    tb = now_s() - t0;
    // C. offsets, lengths and record bytes, per range
    parallel_for(last_range + 1, [&](int t) {
      Range &G = R[t];
      uint64_t o = G.byte_base;
      for (uint64_t i = 0; i < G.keep; i++) {
        const Rec &r = G.recs[i];
        rec_off[G.rec_base + i] = o;
        rec_len[G.rec_base + i] = r.len;
        if (rec_end_block) rec_end_block[G.rec_base + i] = r.done_blk;
        if (r.head)
          for (const Piece &q : G.prefix) {
            copy_nt(rec_buf + o, q.p, q.len);
            o += q.len;
          }
        for (uint32_t k = 0; k < r.npieces; k++) {
          const Piece &q = G.pieces[r.piece0 + k];
          copy_nt(rec_buf + o, q.p, q.len);
          o += q.len;
        }
      }
      _mm_sfence();  // the streamed stores are visible before the call returns
    });
    tc = now_s() - t0;
  };
  // verify and parse side by side; a replay of a few blocks runs both on the
  // calling thread (handing a task to a pool thread costs more than it saves)
  if (n >= 256) {
    parallel_for(2, work);
  } else {
    work(0);
    work(1);
  }
  if (trace)
    std::fprintf(stderr, "[hc_wal_replay] %llu blocks, %d ranges: verify %.3f s, scan+merge %.3f s, "
                 "resolve %.3f s, copy-out %.3f s (from the call start)\n",
                 (unsigned long long)n, T, tv, ta, tb, tc);
  if (vrc < 0) return vrc;
  int code = stop == kErr ? err_code : HC_OK;
  if (first_bad >= 0) {
    const uint64_t B = start_block + (uint64_t)first_bad;
    // the Go loop checks a block's CRC before parsing it: a stop at or after
    // the bad block did not happen, and no record completing there exists
    if (stop == kAll || stop_blk >= B) {
      uint64_t keep = 0;
      for (int t = 0; t <= last_range; t++) {
        const Range &G = R[t];
        uint64_t k = 0;
        while (k < G.keep && G.recs[k].done_blk < B) k++;
        keep += k;
        if (k < G.keep) break;
      }
      count = keep;
      code = HC_ERR_CRC_MISMATCH;
      if (bad_block) *bad_block = (int64_t)B;
      pb = B;
      po = first_bad == 0 ? start_offset : HC_CRC_SIZE;
    }
  }
  *nrec = count;
  *pos_block = pb;
  *pos_offset = po;
  if (pend_pos && code == HC_OK && stop == kAll) pend_pos[0] = pend_blk, pend_pos[1] = pend_hdr;
  return code;
}
