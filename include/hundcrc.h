/*
 * hundcrc.h — C ABI of libhundcrc.so, the MI355X-native batched block-checksum
 * engine that replaces HundDB's utils/crc package.
 *
 * Reference interface replaced (file:line relative to mrsladoje/HundDB):
 *   utils/crc/crc_util.go:11-12  BLOCK_SIZE / CRC_SIZE          -> HC_BLOCK_SIZE / HC_CRC_SIZE
 *   utils/crc/crc_util.go:15-17  GetCRC                          -> hc_crc32_ieee
 *   utils/crc/crc_util.go:21-33  AddCRCToBlockData               -> hc_add_crc_block
 *   utils/crc/crc_util.go:41-64  AddCRCsToData                   -> hc_add_crcs (+ hc_add_crcs_size)
 *   utils/crc/crc_util.go:69-74  SizeAfterAddingCRCs             -> hc_size_after_crcs
 *   utils/crc/crc_util.go:79-83  SizeWithoutCRCs                 -> hc_size_without_crcs
 *   utils/crc/crc_util.go:88-100 CheckBlockIntegrity             -> hc_check_block
 *   utils/crc/crc_util.go:106-122 FixLastBlockCRC                -> hc_fix_last_block
 *   lsm/sstable/sstable.go:2287-2420 CheckIntegrity (md5 + merkle_tree) -> hc_md5*, hc_merkle_* (row f4)
 * New batched entries (the GPU hot path) for the per-block loops of
 *   lsm/block_manager/block_manager.go:203-235 (ReadFromDisk verify loop),
 *   lsm/wal/wal.go:260-271,362-406 (flushBlock / recoverMemtable),
 *   lsm/sstable/sstable.go:660-887 (serialize -> AddCRCsToData).
 *
 * Conventions
 *   - A "block" is a byte range [off, off+len) whose first 4 bytes hold the
 *     little-endian CRC-32/IEEE (Go crc32.ChecksumIEEE) of bytes [4, len).
 *   - All pointers are borrowed for the duration of the call only (the cgo
 *     pointer rule); the library never retains or frees caller memory.
 *   - Host entries (no _dev_) take host pointers, copy through library-owned
 *     pinned staging and are synchronous.  _dev_ entries take device pointers
 *     and a hipStream_t (passed as void*; NULL = HIP's legacy default stream
 *     of the device, one per device and shared by every host thread -- the
 *     library relies on that ordering for the workspace it keeps across NULL-
 *     stream calls; it is built without -fgpu-default-stream=per-thread) and
 *     are asynchronous on that stream.
 *   - Every function is re-entrant and thread-safe.  Shared state: the lazily
 *     initialised per-device constant tables and the bounded pool of host-batch
 *     pipelines (hc_host_pipelines).
 *   - Return codes: >= 0 success / Go-level result; < 0 library error.
 *     No C++ exception ever crosses this ABI.
 */
#ifndef HUNDCRC_H
#define HUNDCRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HC_BLOCK_SIZE 4096u /* crc_util.go:11 (typed uint64 in Go) */
#define HC_CRC_SIZE 4u      /* crc_util.go:12 (untyped constant in Go) */

/* Go-level results (mapped by hc_strerror to the exact errors.New texts) */
#define HC_OK 0
#define HC_ERR_INVALID_BLOCK 1 /* "invalid block data"                            crc_util.go:90  */
#define HC_ERR_CRC_MISMATCH 2  /* "CRC mismatch in block"                         crc_util.go:96  */
#define HC_ERR_TOO_SHORT 3     /* "data is too short to contain a complete block" crc_util.go:108 */
#define HC_ERR_WAL_FRAGMENT_TYPE 4 /* "unknown fragment type"                     wal.go:451      */
#define HC_ERR_WAL_TRUNCATED 5     /* a WAL header/payload runs past its block (Go panics there) */
/* library errors */
#define HC_E_ARG -1     /* invalid argument (null pointer, bad size, capacity too small) */
#define HC_E_HIP -2     /* a HIP runtime call failed */
#define HC_E_NODEV -3   /* no usable gfx950 device: the batched and device entries fail loudly, never
                         * fall back; the three entries that replace a reference function that cannot
                         * fail there -- hc_add_crcs, hc_read_from_disk[_v], hc_wal_replay[_v] -- finish
                         * on the host path instead (as on HC_E_NOMEM / HC_E_HIP; counted in hc_stats) */
#define HC_E_NOMEM -4   /* device or pinned allocation failed */
#define HC_E_LAYOUT -5  /* device batch violated the layout contract (see hc_dev_*) */

/* Exact Go error text for a Go-level result, or a description of a library error. */
const char *hc_strerror(int code);
/* Library version string and the offload arch the kernels were built for. */
const char *hc_version(void);

/* ---------------- drop-ins for utils/crc (crc_util.go) ---------------- */
/* GetCRC (crc_util.go:15-17): crc32.ChecksumIEEE(p[0:n]); n==0 -> 0. */
uint32_t hc_crc32_ieee(const uint8_t *p, size_t n);
/* AddCRCToBlockData (crc_util.go:21-33): n < 4 -> untouched; else
 * p[0:4] = LE32(ChecksumIEEE(p[4:n])).  In place; returns HC_OK. */
int hc_add_crc_block(uint8_t *p, size_t n);
/* Output length of AddCRCsToData for an n-byte input: ceil(n/4092)*4096. */
size_t hc_add_crcs_size(size_t n);
/* AddCRCsToData (crc_util.go:41-64): chunk src into 4092-byte payloads, each
 * in a zeroed 4096-byte block with its CRC in bytes [0:4).  dst is caller
 * memory of >= hc_add_crcs_size(n) bytes (Go: make([]byte, ...)).  Returns the
 * number of bytes written, or (size_t)-1 only if dst_cap is too small (or a
 * pointer is NULL).  Outputs of at least HC_ADD_CRCS_GPU_MIN_BLOCKS blocks
 * (the measured GPU/host crossover) are CRC'd in one GPU batch;
 * when that batch cannot run or fails (no gfx950, HC_E_NOMEM, HC_E_HIP) the
 * CRCs are finished on the host path and the event is counted in hc_stats():
 * the Go function cannot fail, so neither can this.  Only HC_FORCE_GPU=1 (test
 * mode) returns (size_t)-1 for a failed GPU batch. */
size_t hc_add_crcs(const uint8_t *src, size_t n, uint8_t *dst, size_t dst_cap);
/* SizeAfterAddingCRCs (crc_util.go:69-74), float64-ceil semantics. */
uint64_t hc_size_after_crcs(uint64_t n);
/* SizeWithoutCRCs (crc_util.go:79-83), float64-ceil, uint64 wrap for 0<n<4. */
uint64_t hc_size_without_crcs(uint64_t n);
/* CheckBlockIntegrity (crc_util.go:88-100): HC_OK, HC_ERR_INVALID_BLOCK (n<4)
 * or HC_ERR_CRC_MISMATCH. */
int hc_check_block(const uint8_t *p, size_t n);
/* FixLastBlockCRC (crc_util.go:106-122): n < 4096 -> HC_ERR_TOO_SHORT; else
 * restamps the last complete 4096-byte block.  In place. */
int hc_fix_last_block(uint8_t *p, size_t n);

/* ---------------- batched, host-resident (GPU) ---------------- */
/* Block i is base[off[i] .. off[i]+len[i]).  off==NULL -> off[i] = i*stride;
 * len==NULL -> len[i] = ulen.  Blocks shorter than 4 bytes get crc 0 and, for
 * verify, count as bad ("invalid block data").  Any lengths/alignments are
 * accepted; 16-byte-aligned blocks whose length is a multiple of 1024 take the
 * streaming kernel, all others the general kernel (device entries: uniform
 * batches of other shapes may take the message stream). */
int hc_crc32_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                    uint64_t stride, uint32_t ulen, uint64_t nblocks, uint32_t *crc_out);
/* Batched CheckBlockIntegrity.  bad_bitmap (optional, ceil(n/32) uint32 words,
 * bit i%32 of word i/32) marks failing blocks; *first_bad = lowest failing
 * index or -1.  Returns HC_OK if every block passes, HC_ERR_CRC_MISMATCH or
 * HC_ERR_INVALID_BLOCK for the first failing block's reason, < 0 on error. */
int hc_verify_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint64_t stride, uint32_t ulen, uint64_t nblocks, uint32_t *bad_bitmap,
                     int64_t *first_bad);
/* Batched AddCRCToBlockData: stamps every block in place. */
int hc_stamp_blocks(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                    uint32_t ulen, uint64_t nblocks);
/* GetCRC over variable-length messages base[off[i] .. off[i]+len[i]) (whole
 * message, no 4-byte header skipped), e.g. per-record CRCs. */
int hc_crc32_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                      uint64_t nmsgs, uint32_t *crc_out);

/* ---------------- several GPUs in one process ---------------- */
/* Shard plan: contiguous block-index ranges [bounds[d], bounds[d+1]) for ndev
 * GPUs (bounds has ndev+1 entries, bounds[0] = 0, bounds[ndev] = nblocks).
 * len == NULL: by count, bounds[d] = nblocks*d/ndev; else balanced by bytes,
 * bounds[d] = the first block whose byte prefix sum reaches total*d/ndev.  The
 * same plan as hunddb_amd/shard.py (index_range / byte_balanced_bounds). */
int hc_shard_plan(uint64_t nblocks, const uint32_t *len, int ndev, uint64_t *bounds);
/* hc_crc32_blocks / hc_verify_blocks / hc_stamp_blocks over several GPUs: shard d
 * (blocks [bounds[d], bounds[d+1]) of the plan, bounds == NULL: hc_shard_plan)
 * runs on devices[d] through its own host pipeline on its own thread, so each
 * GPU's PCIe link carries its shard.  Outputs as in the one-GPU entries
 * (bad_bitmap / first_bad over the whole batch).  A device may appear more than
 * once.  Returns the first failing shard's error, else as the one-GPU entry. */
int hc_multi_crc32_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                          uint32_t ulen, uint64_t nblocks, uint32_t *crc_out, int ndev, const int *devices,
                          const uint64_t *bounds);
int hc_multi_verify_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                           uint32_t ulen, uint64_t nblocks, uint32_t *bad_bitmap, int64_t *first_bad, int ndev,
                           const int *devices, const uint64_t *bounds);
int hc_multi_stamp_blocks(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t ulen,
                          uint64_t nblocks, int ndev, const int *devices, const uint64_t *bounds);

/* ---------------- batched, device-resident (GPU) ---------------- */
/* As above with device pointers (base, off, len, outputs) on `device`,
 * asynchronous on `stream` (hipStream_t).  crc_out, bad_bitmap and first_bad
 * are each optional (NULL); bad_bitmap must be zeroed and *first_bad set to
 * INT64_MAX by the caller (hc_dev_verify_prepare does both).  `flags`: see
 * HC_F_*.  Returns HC_OK once the work is enqueued. */
#define HC_F_STAMP 1u /* also write each block's CRC into its bytes [0:4) */
#define HC_F_MESSAGES 2u /* whole-message CRC (no 4-byte header skipped) */
int hc_dev_crc32_blocks(int device, const void *base, const uint64_t *off, const uint32_t *len,
                        uint64_t stride, uint32_t ulen, uint64_t nblocks, uint32_t *crc_out,
                        uint32_t *bad_bitmap, int64_t *first_bad, uint32_t flags,
                        void *stream);
/* One shard of a device-resident batch: its blocks, outputs and stream live on
 * `device` (off/len/outputs indexed from the shard's first block). */
typedef struct hc_dev_shard {
  int device;
  const void *base;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride;
  uint32_t ulen;
  uint64_t nblocks;
  uint32_t *crc_out;
  uint32_t *bad_bitmap;
  int64_t *first_bad;
  void *stream;
} hc_dev_shard;
/* hc_dev_crc32_blocks on every shard (each GPU its own shard of a batch,
 * no exchange between them); enqueued on each shard's stream,
 * no synchronisation.  Returns HC_OK once all are enqueued, else the first
 * failing shard's error (shards before it are enqueued). */
int hc_dev_multi_crc32_blocks(const hc_dev_shard *shards, int nshards, uint32_t flags);
/* lsm/block_manager/block_manager.go:189-242 ReadFromDisk, minus the file I/O
 * (row f1): `blocks` holds the blocks from index start_offset/block_size on, as
 * the caller read them (`avail` bytes; past that a block reads as zeros, like
 * readBlockFromDisk's short read).  Every block the loop touches is verified in
 * ONE batch (GPU from HC_READ_GPU_MIN_BLOCKS = 1024, host CPU below), the
 * payload bytes [blockOffset:] of each are copied to out (size bytes; with the
 * GPU batch the copy runs on HC_COPY_THREADS threads while the batch verifies),
 * and *final_offset = SizeAfterAddingCRCs(SizeWithoutCRCs(start_offset) + size).
 * Returns HC_OK or HC_ERR_CRC_MISMATCH with *bad_block = the index (relative to
 * `blocks`) of the first failing block -- the one the Go loop would stop at;
 * then `out` holds unspecified bytes (Go returns no data). */
int hc_read_from_disk(const uint8_t *blocks, uint64_t avail, uint32_t block_size, uint64_t start_offset,
                      uint64_t size, uint8_t *out, uint64_t *final_offset, int64_t *bad_block);
/* Number of blocks ReadFromDisk(start_offset, size) touches (the loop of
 * block_manager.go:203-235 with its CRC-field skip at :195-197). */
uint64_t hc_read_blocks_touched(uint32_t block_size, uint64_t start_offset, uint64_t size);
/* hc_read_from_disk with the block cache's verified bits (row f1): `verified`
 * (optional; ceil(k/32) words, k = hc_read_blocks_touched, bit i = block i
 * relative to `blocks`) marks blocks the caller already verified -- an LRU
 * cache entry whose bytes were CRC-checked and that no caller can have
 * changed since (block_manager.go:72-114; lru_cache.go:20-65; the rule is in
 * INTEGRATION.md section 3) -- and they are NOT hashed again.  On return the bits of every block that
 * this call verified clean are set too, so the cache can record them.
 * *hashed (optional) = blocks whose CRC this call computed. */
int hc_read_from_disk_v(const uint8_t *blocks, uint64_t avail, uint32_t block_size, uint64_t start_offset,
                        uint64_t size, uint32_t *verified, uint8_t *out, uint64_t *final_offset, int64_t *bad_block,
                        uint64_t *hashed);

/* WAL recovery (lsm/wal/wal.go:362-455 recoverMemtable + processBlockForRecovery,
 * row f3) over nblocks written WAL blocks of block_size bytes (every log's
 * written blocks back to back), starting at (start_block, start_offset).
 * All blocks are verified in ONE batch (GPU from HC_WAL_GPU_MIN_BLOCKS = 1024
 * blocks), then parsed:
 * FULL payloads and reassembled FIRST/MIDDLE/LAST fragments are the records
 * (the bytes record.Deserialize receives), copied back to back into rec_buf
 * with rec_off/rec_len.  One call = one memtable: max_records plays
 * memtable.IsFull (0 = never) and, as in Go, the next call starts at the
 * NEXT block.  Returns HC_OK, HC_ERR_CRC_MISMATCH (*bad_block = absolute
 * block index; the records before it are returned), HC_ERR_WAL_FRAGMENT_TYPE
 * or HC_ERR_WAL_TRUNCATED.  If rec_buf_cap / rec_slots run out first, it
 * returns HC_OK with *pos_* at the first record that did not fit (resume
 * there); rec_buf of nblocks*block_size bytes always suffices. */
int hc_wal_replay(const uint8_t *blocks, uint64_t nblocks, uint32_t block_size, uint64_t start_block,
                  uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t rec_buf_cap,
                  uint64_t *rec_off, uint64_t *rec_len, uint64_t rec_slots, uint64_t *nrec, uint64_t *pos_block,
                  uint64_t *pos_offset, int64_t *bad_block);
/* hc_wal_replay plus two optional outputs for callers that replay a long WAL
 * in windows and decide memtable.IsFull themselves (it depends on distinct
 * keys: lsm/memtable skip_list.go:418, btree.go:169, hashmap.go:332):
 *  - rec_end_block (rec_slots entries): the absolute block in which record i
 *    completes (its FULL or LAST fragment).  Replay with max_records = 0, Put
 *    the records in order, and when the memtable fills on record i resume
 *    where wal.go:392-397 does: block rec_end_block[i] + 1, offset CRC_SIZE.
 *  - pend_pos (2 entries): when the call parsed every block without error
 *    (HC_OK, no capacity or max_records stop), the (block, header offset) at
 *    which the fragments still pending at the end start -- the next window
 *    starts there so a record split across windows is rebuilt whole -- or
 *    (UINT64_MAX, 0) when nothing is pending. */
int hc_wal_replay_v(const uint8_t *blocks, uint64_t nblocks, uint32_t block_size, uint64_t start_block,
                    uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t rec_buf_cap,
                    uint64_t *rec_off, uint64_t *rec_len, uint64_t *rec_end_block, uint64_t rec_slots,
                    uint64_t *nrec, uint64_t *pos_block, uint64_t *pos_offset, int64_t *bad_block,
                    uint64_t *pend_pos);

/* Fused AddCRCsToData on device memory (utils/crc/crc_util.go:41-64): frame the
 * n-byte payload src (any alignment) into ceil(n/4092) zero-padded 4096-byte
 * blocks at dst (16-byte aligned, >= hc_add_crcs_size(n) bytes) and stamp each
 * block's CRC in bytes 0..3; crc_out (optional) receives the per-block CRCs.
 * One read of src and one write of dst (kernel k_frame).  HC_E_LAYOUT if dst
 * is not 16-byte aligned.  n == 0 writes nothing (Go returns an empty slice). */
int hc_dev_add_crcs(int device, const void *src, uint64_t n, void *dst, uint32_t *crc_out,
                    void *stream);
/* Batched ReadFromDisk on device memory (block_manager.go:203-235, row f1):
 * verify nblocks blocks of block_size (4096, 8192 or 16384) bytes at `blocks`
 * (16-byte aligned) like CheckBlockIntegrity, and write each block's payload
 * block[4:] back to back at payload_out (nblocks * (block_size - 4) bytes).
 * Verification outputs as in hc_dev_crc32_blocks (crc_out = computed CRCs;
 * bad_bitmap/first_bad prepared by hc_dev_verify_prepare).  Kernel k_unframe:
 * one read of the blocks, one write of the payload.  HC_E_LAYOUT for another
 * block size or an unaligned `blocks`. */
int hc_dev_read_blocks(int device, const void *blocks, uint64_t nblocks, uint32_t block_size,
                       void *payload_out, uint32_t *crc_out, uint32_t *bad_bitmap, int64_t *first_bad,
                       void *stream);
/* Zero a device bitmap of ceil(n/32) words and set *first_bad = INT64_MAX. */
int hc_dev_verify_prepare(int device, uint32_t *bad_bitmap, int64_t *first_bad,
                          uint64_t nblocks, void *stream);
/* Fill a device buffer with the seeded synthetic workload: block i occupies
 * [off[i], off[i]+len[i]) (or i*stride / ulen), 64-bit word w of block i =
 * splitmix64(seed, i, w) (see oracle/hc_oracle.c oc_splitmix64). */
int hc_dev_fill_blocks(int device, void *base, const uint64_t *off, const uint32_t *len,
                       uint64_t stride, uint32_t ulen, uint64_t nblocks, uint64_t seed,
                       void *stream);
/* The same for a shard of a global batch: buffer block i gets the bytes of
 * global block first_block + i (word w = splitmix64(seed, first_block + i, w)),
 * so N ranks filling index ranges hold exactly the one-GPU batch. */
int hc_dev_fill_range(int device, void *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                      uint32_t ulen, uint64_t first_block, uint64_t nblocks, uint64_t seed, void *stream);

/* ---- row f4: Merkle/MD5 integrity of SSTable data ----------------------------
 * lsm/sstable/sstable.go:2287-2420 CheckIntegrity: md5.Sum of every record
 * (:2358), merkle_tree.NewMerkleTree(leaves, true) (:2368,
 * merkle_tree.go:36-81), Deserialize of the stored tree and Validate
 * (merkle_tree.go:115-147,192-226).  Digests are the 16 bytes md5.Sum returns. */
/* md5.Sum(p[0:n]) on the host CPU (one record or one node). */
void hc_md5(const uint8_t *p, size_t n, uint8_t out[16]);
/* md5.Sum of every message base[off[i] .. off[i]+len[i]) into out16 + 16*i:
 * one GPU batch (the leaves of CheckIntegrity).  HC_E_NODEV without a GPU. */
int hc_md5_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out16);
/* Device form: message i = base[off(i) .. +len(i)) (off/len arrays or
 * i*stride / ulen, as hc_dev_crc32_blocks), digests into out16 (device,
 * 16-B aligned).  workspace: device memory of hc_md5_workspace_bytes(n)
 * bytes (the waves' ranges of equal work for off/len batches of 16384 to 32M
 * messages; else 0), or NULL (then allocated per call on `stream`).
 * Kernel k_md5 (lane per message). */
uint64_t hc_md5_workspace_bytes(uint64_t n);
int hc_dev_md5_messages(int device, const void *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                        uint32_t ulen, uint64_t n, uint8_t *out16, void *workspace, void *stream);
/* Entries of the Merkle level layout for n leaves: level 0 = the leaves, each
 * level with an odd number (> 1) of nodes followed by its zero padding node
 * (merkle_tree.go:60-66), then the parent levels up to the root (the last
 * entry).  n == 0: one entry, md5.Sum([]byte{}) (merkle_tree.go:37). */
uint64_t hc_merkle_nodes(uint64_t n);
/* NewMerkleTree(leaves, hashedAlready=true) as level arrays: copies the n leaf
 * digests into levels16 (hc_merkle_nodes(n)*16 bytes, may alias leaves16) and
 * fills the padding nodes and parents (GPU from 65536 leaves, host below). */
int hc_merkle_levels(const uint8_t *leaves16, uint64_t n, uint8_t *levels16);
/* Device form: levels16 (device, 16-B aligned) already holds the n leaves in
 * its first entries (e.g. from hc_dev_md5_messages); kernel k_merkle_level
 * per level. */
int hc_dev_merkle_levels(int device, uint8_t *levels16, uint64_t n, void *stream);
/* MerkleTree.Serialize() (merkle_tree.go:173-187): DFS pre-order, 16 bytes
 * per node, into out (cap bytes); *nbytes = hc_merkle_nodes(n)*16.  out ==
 * NULL: size query only. */
int hc_merkle_serialize(const uint8_t *levels16, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *nbytes);
/* tree.Validate(merkle_tree.Deserialize(stored)) exactly as CheckIntegrity
 * calls it (sstable.go:2394-2411): *valid = 1 when the roots agree; else the
 * mismatched leaf pair DeepValidate reports (*nmism = 0 or 1: Deserialize
 * builds a left chain, so at most one pair), built-tree hash / stored hash.
 * stored_len must be a positive multiple of 16 (Go panics otherwise). */
int hc_merkle_validate(const uint8_t *levels16, uint64_t n, const uint8_t *stored, uint64_t stored_len, int *valid,
                       uint8_t *mism_built16, uint8_t *mism_stored16, uint64_t *nmism);

/* Per-launch accounting of the last device call on this thread (for the
 * roofline): kernel name, number of blocks routed to the streaming kernel and
 * to the general kernel, and algorithmic bytes (sum of block lengths). */
typedef struct {
  const char *kernel;
  uint64_t fast_blocks, general_blocks, bytes;
  uint32_t grid, block_threads, lds_bytes;
} hc_launch_info;
int hc_last_launch(hc_launch_info *info);

/* Copy the host-built constant image the kernels use (DESIGN.md "Tables")
 * into out (returns HC_OK) or, if cap is too small, return its size. */
int hc_debug_tables(void *out, size_t cap);

/* How this thread's last device batch of whole messages was hashed: 1 by the
 * packed-record stream (k_seg_*) as records back to back, 4 by
 * the same stream as sorted records with gaps of at most 64 B between them, 2
 * as sorted records with wider gaps (zeroed in the stream), 3 by k_crc_grp
 * (the stream's fallback for aligned 4 KiB-multiple records out of order), 0
 * by k_crc_any on the device or not offered to the stream; plus 8 when the
 * records were listed out of order and the stream ran over their sorted view
 * (from HC_SEG_SORT_MIN records); synchronizes that device
 * (tests and tools only). */
int hc_debug_seg_taken(void);
/* The stream kernel's phase clock for this thread's last batch on the stream
 * (DESIGN.md 4.2b): 16 s_memrealtime stamps (100 MHz) of workgroup 0 -- [0]
 * start, [1] prologue done, [2] the sort's key range and residency check,
 * [3..7] its barriers after A1, A2, A3, B, P5, [10] P6, [14] / [15] the sorted
 * view's stream body start / end (stale entries when no sort ran).
 * Synchronizes that device (tools only). */
int hc_debug_seg_prof(uint64_t *out16);

/* The library reads its HC_* settings from the environment once, at the first
 * call that needs one (a getenv racing with a Go os.Setenv would be a data
 * race): HC_DEVICE, HC_SEG_MIN_MSGS, HC_COPY_THREADS, HC_WAL_MIN_RANGE,
 * HC_ADD_CRCS_GPU_MIN_BLOCKS, HC_READ_GPU_MIN_BLOCKS, HC_WAL_GPU_MIN_BLOCKS,
 * HC_FORCE_GPU, HC_INJECT_FAIL, HC_SEG_GRP_MIN, HC_SEG_MIN_BLOCKS, HC_SEG_SORT_MIN,
 * HC_SEG_SYNC_SPINS, HC_SEG_SORT_UC, HC_SEG_LG_CHUNK.  hc_debug_set changes one of them afterwards
 * (tests and tools); value NULL restores the compiled default.  HC_OK, or
 * HC_E_ARG for an unknown name.
 * HC_INJECT_FAIL (test hook) accepts "add_crcs", "read_from_disk" or
 * "wal_replay": that GPU batch reports HC_E_HIP and the host path finishes it;
 * "<site>:nomem" reports HC_E_NOMEM instead; "<site>:<other>" keeps HC_E_HIP
 * (with a note on stderr); an unknown site injects nothing. */
int hc_debug_set(const char *name, const char *value);

/* Number of visible gfx950 devices (0 if none; never initialises a context
 * on a machine without GPUs). */
int hc_device_count(void);
/* Host-batch pipelines alive in this process (pinned staging + device buffers
 * + streams).  Host entries lease one per call from a pool of at most
 * HC_MAX_PIPES (default 4) per device; further concurrent callers wait for a free one. */
int hc_host_pipelines(void);

/* Process-wide event counters (monotonic since load or hc_stats_reset).
 * The three host entries that replace a reference function with a host path
 * of its own -- AddCRCsToData (hc_add_crcs), ReadFromDisk (hc_read_from_disk*)
 * and WAL recovery (hc_wal_replay*) -- run a GPU batch above their threshold
 * and, when that batch cannot run or fails, finish on the host path instead
 * of failing where the reference cannot (only HC_FORCE_GPU returns the error).
 *   add_crcs_gpu / read_gpu / wal_gpu: calls whose batch ran on the GPU;
 *   add_crcs_host_small: AddCRCsToData outputs below the GPU threshold;
 *   add_crcs_host_nodev / nodev_host: GPU batch skipped, no usable gfx950
 *     (AddCRCsToData / the other two);
 *   *_gpu_fallback: GPU batch failed (HC_E_NOMEM, HC_E_HIP), finished on the
 *     host; last_fallback_error = the last such batch's HC_E_* code. */
typedef struct hc_stats_t {
  uint64_t add_crcs_gpu;
  uint64_t add_crcs_host_small;
  uint64_t add_crcs_host_nodev;
  uint64_t add_crcs_gpu_fallback;
  int64_t last_fallback_error;
  uint64_t read_gpu;
  uint64_t read_gpu_fallback;
  uint64_t wal_gpu;
  uint64_t wal_gpu_fallback;
  uint64_t nodev_host;
} hc_stats_t;
int hc_stats(hc_stats_t *out);
void hc_stats_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* HUNDCRC_H */
