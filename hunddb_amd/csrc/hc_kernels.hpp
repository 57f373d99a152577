// hc_kernels.hpp — launch interface between the host runtime (hc_api.cpp) and
// the gfx950 kernels (hc_kernels.hip).  No torch types, plain pointers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hc_gf2.hpp"

namespace hc {

enum : uint32_t { kFlagStamp = 1u, kFlagMessages = 2u };

// One batch of blocks (or messages) as the kernels see it.  Block i occupies
// base[off(i) .. off(i)+len(i)) with off(i) = off ? off[i] : i*stride and
// len(i) = len ? len[i] : ulen.
struct Batch {
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride;
  uint32_t ulen;
  uint32_t flags;
  uint64_t nblocks;
  uint32_t *crc_out;              // optional
  uint32_t *bad_bitmap;           // optional (verify)
  unsigned long long *first_bad;  // optional (verify), INT64_MAX when clean
  const DeviceTables *tables;
  // optional (off/len batches): k_crc_grp raises *skip_slot to at least
  // skip_tag (atomic max) when it leaves a block to k_crc_any, and the k_crc_any
  // sweep after it exits at once while *skip_slot < skip_tag.  Tags increase
  // per call, so a slot shared by concurrent calls (or a graph replaying an old
  // tag) can only make a sweep run without need, never skip one that has work.
  unsigned long long *skip_slot;
  uint64_t skip_tag;
};

// Streaming kernel geometry (one workgroup per CU; see DESIGN.md "Kernel").
constexpr int kFastWaves = 16;
constexpr int kFastThreads = kFastWaves * 64;
constexpr uint32_t kLdsMainBytes = 131072;  // 4 row-shift tables x 256 x 32 replicas x 4 B
constexpr uint32_t kLdsS4Bytes = 16384;     // 4 x 256 x 4 replicas x 4 B
constexpr uint32_t kFastLdsBytes = kLdsMainBytes + kLdsS4Bytes;


// Host launchers; return the hipError_t of the launch.
// k_crc_fast: uniform batches only (no off/len arrays), every block 16-B
// aligned with a length that is a positive multiple of 1024 (refused otherwise).
hipError_t launch_fast(const Batch &b, int grid, hipStream_t s);
// k_crc_any.  fast_mask != 0: process only the blocks a streaming kernel
// skipped, i.e. all but the 16-B aligned ones whose length is a positive
// multiple of fast_mask+1 (4095: k_crc_grp).  0: every block.
hipError_t launch_general(const Batch &b, uint32_t fast_mask, int grid, hipStream_t s);
// k_crc_grp: 4 KiB-multiple blocks (uniform, or off/len with device-side
// routing of the others to k_crc_any with fast_mask 4095), per-workgroup
// dynamic hand-out of chunked blocks.
bool grp_xcd(uint32_t block_bytes, int grid, uint64_t nblocks);
uint32_t grp_lg_chunk(uint64_t nblocks, int grid, uint32_t block_bytes);
hipError_t launch_grp(const Batch &b, int grid, hipStream_t s);
// (launch_frame and launch_unframe refuse grids of more than kMaxGridWgs
// 256-thread workgroups: HIP's limit is gridDim.x * blockDim.x < 2^32.)
constexpr uint64_t kMaxGridWgs = 0xFFFFFFFFull / 256;
// Fused AddCRCsToData: frame n payload bytes into (n+4091)/4092 stamped 4096-B
// blocks in ONE launch of k_frame (its workgroup 0 does the two edge blocks,
// every other wave one interior block; `grid` is unused).
constexpr uint32_t HC_FRAME_BLOCK = 4096;
hipError_t launch_frame(const uint8_t *src, uint64_t n, uint8_t *dst, uint32_t *crc_out,
                        const DeviceTables *tables, int grid, hipStream_t s);
constexpr uint32_t kLaneQWords = 8 * kLanes * 4;  // k_frame / k_unframe: LDS copy of DeviceTables::lane_q

// Geometry of the framing kernels (256-thread, 4-wave workgroups):
//   * k_frame and k_unframe at 4 KiB: a workgroup's four waves take blocks
//     kFrameSpread apart, kFrameSpread neighbouring workgroups one contiguous
//     run of 4 x kFrameSpread blocks.  kFrameSpread is a multiple of 4, so b mod
//     4 -- the 4092-B stride's misalignment -- is one per workgroup.  Spreads 4
//     / 8 / 16 / 32 measured (profiles/r3/kframe4/): 8 is the fastest.
//   * k_unframe at 8 / 16 KiB: one 4 KiB group per wave, a block's groups in
//     one workgroup; 8 KiB blocks in runs of 8 over 4 workgroups (one output
//     alignment per workgroup), 16 KiB blocks one per workgroup.
constexpr uint32_t kFrameSpread = 8;
inline uint64_t unframe_grid(uint64_t nblk, uint32_t lg_groups) {
  return lg_groups == 0 ? kFrameSpread * ((nblk + 4 * kFrameSpread - 1) / (4 * kFrameSpread))
         : lg_groups == 1 ? 4 * ((nblk + 7) / 8)
                          : nblk;
}
// Batched ReadFromDisk: verify nblk blocks of 4096 << lg_groups bytes at `blocks`
// (16-B aligned) and write their payloads back to back at `out`.  Its own grid
// (unframe_grid: 4-wave workgroups, one 4 KiB group per wave).  Refused
// (hipErrorInvalidValue) when the grid's work-items would pass 2^32 - 1.
hipError_t launch_unframe(const uint8_t *blocks, uint64_t nblk, uint32_t lg_groups, uint8_t *out,
                          uint32_t *crc_out, uint32_t *bad_bitmap, unsigned long long *first_bad,
                          const DeviceTables *tables, hipStream_t s);
// synthetic workload: buffer block i = block first + i of the seeded batch
hipError_t launch_fill(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                       uint32_t ulen, uint64_t n, uint64_t seed, int grid, hipStream_t s, uint64_t first = 0);
// Row f4 (hc_md5.hip): MD5 of each message (16-B digests at out16; workspace
// = md5_workspace_bytes(n) bytes of device memory: tail slots + schedule), and
// the Merkle levels above n leaves stored at levels16 (layout:
// hc_merkle_nodes in include/hundcrc.h).
uint64_t md5_workspace_bytes(uint64_t n);
hipError_t launch_md5(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t ulen,
                      uint64_t n, uint8_t *workspace, uint8_t *out16, int cus, hipStream_t s);
hipError_t launch_merkle_levels(uint8_t *levels16, uint64_t n, hipStream_t s);
// Whole-message batches (HC_F_MESSAGES) as one stream over their span
// (k_seg_*, hc_kernels.hip): records back to back (off[i+1] = off[i] +
// len[i]), or sorted with gaps of at most a quarter of the payload between
// them.  max_units bounds the span's 16 KiB units (seg_max_units of a byte
// bound on the span); ws holds seg_workspace_bytes(n, max_units) bytes.  A
// batch the stream refuses (out of order or overlapping, larger than the
// bound, records under ~64 B or over 16 MiB) sets ws[0] on the device and
// k_seg_combine runs k_crc_any's work over it in the same launch; from grp_min
// records on, a batch of aligned 4 KiB-multiple records goes to k_crc_grp in
// any layout, launched after the combine, which exits at once unless ws[0] says so.
// An unsorted batch of at least sort_min records (round 6) is
// sorted by record offset inside k_seg_stream (grid barriers; its workspace is
// the sort part of seg_workspace_bytes(n, max_units, true)) and streamed in
// that order; k_seg_combine writes each word through the permutation.
// sort_min 0: never (the workspace may then be seg_workspace_bytes(n, mu)).
uint64_t seg_max_units(uint64_t span_bound);
uint64_t seg_workspace_bytes(uint64_t n, uint64_t max_units, bool sort = false);
constexpr uint64_t kSegGrpFallbackMin = 1ull << 18;  // grp_min's default (HC_SEG_GRP_MIN)
// sort_min's default (HC_SEG_SORT_MIN): the sorted view's fixed cost (its grid barriers,
// ~170 us) against k_crc_any's work on permuted config-5 records broke even near 2^18
// records (0.594 vs 0.585 ms; 16k: 0.257 vs 0.085, 1M: 1.71 vs 2.02; profiles/r6/r6bb/)
constexpr uint64_t kSegSortMin = 1ull << 18;
// taken (optional, device word): 1 packed, 2 gapped, 3 k_crc_grp fallback,
// 4 small gaps, 0 k_crc_any fallback; | 8 when the stream ran on the sorted view.
// sync_spins bounds the sort's first grid barrier, the check that the grid is
// resident (polls; a grid that is not: no sort, k_crc_any's work).
constexpr uint32_t kSegSyncSpinsDefault = 1u << 17;
// sort_uc (test hook; 0 = the default, 32768) bounds the units of one coarse
// bucket of the sort, so that small spans can run several buckets a workgroup.
// the stream's chunk slot: 2^3 units of 16 KiB (HC_SEG_LG_CHUNK; round 6 sweep)
constexpr uint32_t kSegLgChunk = 3;
hipError_t launch_seg(const Batch &b, const SegTables *st, uint32_t *ws, uint64_t max_units, int grid, hipStream_t s,
                      uint32_t *taken = nullptr, uint64_t grp_min = kSegGrpFallbackMin, uint64_t sort_min = 0,
                      uint32_t sync_spins = kSegSyncSpinsDefault, uint32_t sort_uc = 0, uint32_t lg_chunk = kSegLgChunk);
// A uniform block batch (no off/len arrays) that k_crc_grp refuses (lengths not
// a 4 KiB multiple, or not 16-B aligned), ulen >= 4, stride >= ulen: its
// messages block[4:ulen] written out as off/len arrays, launch_seg over them
// (they lie stride - ulen + 4 bytes apart: the small-gap mode), then the
// blocks' verify / stamp outputs from the message CRCs.  ws holds
// seg_block_workspace_bytes(n, max_units, !b.crc_out) bytes.
uint64_t seg_block_workspace_bytes(uint64_t n, uint64_t max_units, bool crc_words);
// the sort's phase clock (hc_debug_seg_prof): 16 s_memrealtime stamps (100 MHz) of workgroup 0
hipError_t seg_prof_read(uint64_t *out16);
hipError_t launch_seg_blocks(const Batch &b, const SegTables *st, uint32_t *ws, uint64_t max_units, int grid,
                             hipStream_t s, uint32_t *taken = nullptr);
hipError_t launch_verify_prepare(uint32_t *bitmap, unsigned long long *first_bad, uint64_t n,
                                 hipStream_t s);

}  // namespace hc
