/*
 * hc_oracle.h — CPU oracle for the HundDB utils/crc hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under hunddb_amd/ links, includes or calls
 * this code.  It is used by tests/ (as the checker), by
 * __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline leg
 * (the reference Go CPU path restated in C and timed on the host cores).
 *
 * What it restates:
 *   - Go stdlib hash/crc32 (go 1.23.2, pinned by /root/reference/go.mod:3; the
 *     package is NOT vendored under /root/reference) as called by
 *     utils/crc/crc_util.go:16 and :94 (crc32.ChecksumIEEE).  Three forms of
 *     its published algorithm family are restated: the bit-serial definition
 *     of CRC-32/ISO-HDLC, Go's simpleUpdate (Sarwate byte table), Go's
 *     slicingUpdate (slicing-by-8, slicing8Cutoff = 16) and Go's amd64
 *     archUpdateIEEE (PCLMULQDQ 4x128-bit folding for the 16-byte-aligned
 *     prefix of inputs >= 64 bytes, slicing-by-8 tail).
 *   - Every function of utils/crc/crc_util.go:10-122, with its edge cases,
 *     error strings, constant 4096 framing and float64 ceil size math.
 *   - The WAL block framing of lsm/wal/wal.go:177-283 + wal_header.go:5-77
 *     + model/record/record.go:85-119 (config 5 workload generator).
 *   - Row f4: MD5 (Go crypto/md5, RFC 1321) and lsm/sstable/merkle_tree
 *     (oc_merkle.c), pinned by the RFC 1321 suite and merkle_tree_test.go.
 *
 * Pinning: tests/golden/ (JSON fixtures), generated in the build container by
 * tests/golden/gen_golden.py with Python zlib.crc32 (zlib 1.2.11, the same
 * CRC-32/ISO-HDLC function).  The reference has no CRC golden vectors of its
 * own; see DESIGN.md "Oracle".
 */
#ifndef HC_ORACLE_H
#define HC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- CRC-32/ISO-HDLC arithmetic (Go hash/crc32, IEEE) ---------------- */
uint32_t oc_crc32_bitwise(uint32_t crc, const uint8_t *p, size_t n);  /* definition */
uint32_t oc_crc32_sarwate(uint32_t crc, const uint8_t *p, size_t n);  /* Go simpleUpdate */
uint32_t oc_crc32_slicing8(uint32_t crc, const uint8_t *p, size_t n); /* Go slicingUpdate */
uint32_t oc_crc32_go_amd64(uint32_t crc, const uint8_t *p, size_t n); /* Go archUpdateIEEE */
int oc_have_pclmul(void);
/* crc32.ChecksumIEEE(p) == oc_checksum_ieee(p, n) */
uint32_t oc_checksum_ieee(const uint8_t *p, size_t n);

/* ---- utils/crc/crc_util.go restated ----------------------------------- */
#define OC_BLOCK_SIZE 4096u
#define OC_CRC_SIZE 4u
/* error codes; strings identical to the Go errors.New texts */
#define OC_OK 0
#define OC_ERR_INVALID_BLOCK 1   /* "invalid block data"                            */
#define OC_ERR_CRC_MISMATCH 2    /* "CRC mismatch in block"                         */
#define OC_ERR_TOO_SHORT 3       /* "data is too short to contain a complete block" */
#define OC_ERR_WAL_FRAGMENT_TYPE 4 /* "unknown fragment type" (wal.go:451)            */
#define OC_ERR_WAL_TRUNCATED 5   /* header/payload past the block end (Go panics)   */
const char *oc_strerror(int code);
uint32_t oc_get_crc(const uint8_t *p, size_t n);                      /* :15-17 */
void oc_add_crc_to_block_data(uint8_t *p, size_t n);                  /* :21-33 */
size_t oc_add_crcs_to_data(const uint8_t *src, size_t n, uint8_t *dst); /* :41-64, returns len */
uint64_t oc_size_after_adding_crcs(uint64_t n);                       /* :69-74 */
uint64_t oc_size_without_crcs(uint64_t n);                            /* :79-83 */
int oc_check_block_integrity(const uint8_t *p, size_t n);             /* :88-100 */
int oc_fix_last_block_crc(uint8_t *p, size_t n);                      /* :106-122 */

/* lsm/block_manager/block_manager.go:189-242 ReadFromDisk over an in-memory
 * block image starting at block start_offset/block_size (avail bytes, zeros
 * after); returns OC_OK or the CheckBlockIntegrity code, *bad_block = relative
 * index of the failing block (-1 if none). */
int oc_read_from_disk(const uint8_t *blocks, uint64_t avail, uint32_t block_size, uint64_t start_offset,
                      uint64_t size, uint8_t *out, uint64_t *final_offset, int64_t *bad_block);

/* ---- batches ----------------------------------------------------------- */
/* CRC of blk[4:len] for each block (what CheckBlockIntegrity computes), on
 * nthreads host threads using oc_crc32_go_amd64.  off==NULL => off=i*stride;
 * len==NULL => len=ulen. */
void oc_crc32_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint64_t stride, uint32_t ulen, uint32_t *out, size_t nblocks,
                     int nthreads);
/* CRC of whole messages p[off:off+len] (GetCRC over variable-length records) */
void oc_crc32_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       uint32_t *out, size_t n, int nthreads);

/* ---- synthetic inputs (identical generator in HIP, numpy and here) ----- */
uint64_t oc_splitmix64(uint64_t seed, uint64_t block, uint64_t word);
/* fill len bytes (len % 8 == 0) of block `block` */
void oc_fill_block(uint64_t seed, uint64_t block, uint8_t *dst, size_t len);
/* blocks first .. first+n-1 of a uniform batch, on nthreads threads */
void oc_fill_blocks_mt(uint64_t seed, uint64_t first, uint64_t n, uint64_t block_bytes, uint8_t *dst, int nthreads);
/* block size of block i of the mixed 4/8/16 KiB batch (config 3) */
uint32_t oc_mixed_size(uint64_t seed, uint64_t block);

/* ---- WAL framing (lsm/wal/wal.go:177-283) ------------------------------ */
typedef struct {
  uint64_t records, blocks, refused, fragments;
} oc_wal_stats;
/* Frames `nrec` records whose serialized sizes are given into `bs`-byte WAL
 * blocks exactly as WriteRecord/writeFragmentedRecord/writeToBlock/flushBlock.
 * If dst != NULL it must hold max_blocks*bs bytes; blocks are CRC-stamped
 * (flushBlock's AddCRCToBlockData) unless stamp==0.  Record payload bytes are
 * derived from (seed, record index).  Returns blocks written (stops at
 * max_blocks).  `next_rec` (if non-NULL) receives the first record not framed. */
uint64_t oc_wal_frame(uint64_t seed, const uint32_t *rec_sizes, uint64_t nrec, uint32_t bs,
                      uint8_t *dst, uint64_t max_blocks, int stamp, oc_wal_stats *st,
                      uint64_t *next_rec);
/* WAL recovery, lsm/wal/wal.go:362-455, over nblocks written blocks of bs
 * bytes (all logs back to back), starting at (start_block, start_offset).
 * Emits the serialized records (FULL payloads and reassembled FIRST..LAST
 * fragments) into rec_buf (>= nblocks*bs bytes) with rec_off/rec_len, stops
 * after max_records (memtable.IsFull; 0 = never), and returns OC_OK,
 * OC_ERR_CRC_MISMATCH (*bad_block), OC_ERR_WAL_FRAGMENT_TYPE or
 * OC_ERR_WAL_TRUNCATED.  *pos_* = where the next memtable's replay starts. */
int oc_wal_replay(const uint8_t *blocks, uint64_t nblocks, uint32_t bs, uint64_t start_block,
                  uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t *rec_off,
                  uint64_t *rec_len, uint64_t *nrec, uint64_t *pos_block, uint64_t *pos_offset,
                  int64_t *bad_block);
/* log-uniform serialized record size in [lo, hi] for record i */
uint32_t oc_wal_record_size(uint64_t seed, uint64_t i, uint32_t lo, uint32_t hi);

/* ---- row f4: Merkle/MD5 integrity (oc_merkle.c) ------------------------- */
/* md5.Sum (RFC 1321) */
void oc_md5(const uint8_t *p, size_t n, uint8_t out[16]);
void oc_md5_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint8_t *out, size_t n);
/* NewMerkleTree(leaves, hashedAlready=true) root; n == 0: md5("") */
void oc_merkle_root(const uint8_t *leaves, uint64_t n, uint8_t root[16]);
/* ... .Serialize(): DFS pre-order, 16 B per node; returns bytes (out may be NULL) */
uint64_t oc_merkle_serialize(const uint8_t *leaves, uint64_t n, uint8_t *out);
/* tree(leaves).Validate(Deserialize(stored)): 1 equal roots, 0 not (mismatched
 * leaf pairs, DeepValidate order, into mism1/mism2, up to cap; *nmism = all),
 * -1 when stored is empty (a nil root: Go panics) */
int oc_merkle_validate(const uint8_t *leaves, uint64_t n, const uint8_t *stored, uint64_t stored_len,
                       uint8_t *mism1, uint8_t *mism2, uint64_t cap, uint64_t *nmism);
/* tree(leaves1).Validate(tree(leaves2)), both built (merkle_tree_test.go TestValidate) */
int oc_merkle_validate_trees(const uint8_t *l1, uint64_t n1, const uint8_t *l2, uint64_t n2, uint8_t *mism1,
                             uint8_t *mism2, uint64_t cap, uint64_t *nmism);

#ifdef __cplusplus
}
#endif
#endif
