/*
 * hc_oracle.c — CPU oracle for the HundDB utils/crc hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see hc_oracle.h).  The product (hunddb_amd/) never
 * links or calls this file; tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do, as the checker / the timed reference CPU path.
 *
 * Reference being restated (file:line relative to /root/reference):
 *   utils/crc/crc_util.go:10-122   the drop-in surface (restated 1:1 below)
 *   Go 1.23.2 hash/crc32 (go.mod:3; external, not vendored): ChecksumIEEE,
 *     simpleUpdate, slicingUpdate, amd64 archUpdateIEEE/ieeeCLMUL.  Restated
 *     from the published algorithms (CRC-32/ISO-HDLC; Sarwate; slicing-by-8;
 *     Gopal et al. "Fast CRC Computation for Generic Polynomials Using
 *     PCLMULQDQ", Intel 2009, whose 4x128-bit fold + Barrett reduction Go's
 *     crc32_amd64.s implements).
 *   lsm/wal/wal.go:177-283, wal_header.go:5-77, model/record/record.go:85-119
 *     WAL block framing (config-5 generator).
 */
#include "hc_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

#define POLY_REFLECTED 0xEDB88320u /* CRC-32/ISO-HDLC, reflected */

/* ------------------------------------------------------------------------ */
/* Bit-serial definition: refin/refout, poly 0x04C11DB7, init/xorout ~0.     */
/* Caller passes and receives the *finalised* crc like Go's Update().        */
uint32_t oc_crc32_bitwise(uint32_t crc, const uint8_t *p, size_t n) {
  crc = ~crc;
  for (size_t i = 0; i < n; i++) {
    crc ^= p[i];
    for (int b = 0; b < 8; b++) crc = (crc >> 1) ^ (POLY_REFLECTED & (0u - (crc & 1u)));
  }
  return ~crc;
}

/* Go hash/crc32 tables: simpleMakeTable + slicingMakeTable (8 tables). */
static uint32_t g_tab8[8][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_tables(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (POLY_REFLECTED & (0u - (c & 1u)));
    g_tab8[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = g_tab8[0][i];
    for (int t = 1; t < 8; t++) {
      c = g_tab8[0][c & 0xFF] ^ (c >> 8);
      g_tab8[t][i] = c;
    }
  }
}
static inline void tables(void) { pthread_once(&g_once, init_tables); }

/* Go simpleUpdate (crc32_generic.go): one Sarwate table lookup per byte. */
uint32_t oc_crc32_sarwate(uint32_t crc, const uint8_t *p, size_t n) {
  tables();
  crc = ~crc;
  for (size_t i = 0; i < n; i++) crc = g_tab8[0][(uint8_t)crc ^ p[i]] ^ (crc >> 8);
  return ~crc;
}

static inline uint32_t le32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

/* Go slicingUpdate (crc32_generic.go): slicing-by-8 for len >= 16. */
uint32_t oc_crc32_slicing8(uint32_t crc, const uint8_t *p, size_t n) {
  tables();
  if (n >= 16) {
    crc = ~crc;
    while (n > 8) {
      crc ^= le32(p);
      crc = g_tab8[0][p[7]] ^ g_tab8[1][p[6]] ^ g_tab8[2][p[5]] ^ g_tab8[3][p[4]] ^
            g_tab8[4][crc >> 24] ^ g_tab8[5][(crc >> 16) & 0xFF] ^
            g_tab8[6][(crc >> 8) & 0xFF] ^ g_tab8[7][crc & 0xFF];
      p += 8;
      n -= 8;
    }
    crc = ~crc;
  }
  if (n == 0) return crc;
  return oc_crc32_sarwate(crc, p, n);
}

int oc_have_pclmul(void) {
#if defined(__x86_64__)
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
  return (c & bit_PCLMUL) && (c & bit_SSE4_1);
#else
  return 0;
#endif
}

#if defined(__x86_64__)
/* ieeeCLMUL: 4x128-bit folding over len (>=64, %16==0) bytes; crc is the raw
 * (non-inverted) register.  Constants are x^k mod P, bit-reflected, << 1. */
__attribute__((target("pclmul,sse4.1"))) static uint32_t clmul_fold(uint32_t crc,
                                                                     const uint8_t *p,
                                                                     size_t n) {
  const __m128i r2r1 = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);
  const __m128i r4r3 = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);
  const __m128i r5 = _mm_set_epi64x(0, 0x163cd6124LL);
  const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
  const __m128i rupoly = _mm_set_epi64x(0x1F7011641LL, 0x1DB710641LL);
  __m128i x1 = _mm_loadu_si128((const __m128i *)(p + 0));
  __m128i x2 = _mm_loadu_si128((const __m128i *)(p + 16));
  __m128i x3 = _mm_loadu_si128((const __m128i *)(p + 32));
  __m128i x4 = _mm_loadu_si128((const __m128i *)(p + 48));
  x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
  p += 64;
  n -= 64;
  while (n >= 64) {
    __m128i y1 = _mm_clmulepi64_si128(x1, r2r1, 0x11);
    __m128i y2 = _mm_clmulepi64_si128(x2, r2r1, 0x11);
    __m128i y3 = _mm_clmulepi64_si128(x3, r2r1, 0x11);
    __m128i y4 = _mm_clmulepi64_si128(x4, r2r1, 0x11);
    x1 = _mm_clmulepi64_si128(x1, r2r1, 0x00);
    x2 = _mm_clmulepi64_si128(x2, r2r1, 0x00);
    x3 = _mm_clmulepi64_si128(x3, r2r1, 0x00);
    x4 = _mm_clmulepi64_si128(x4, r2r1, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, y1), _mm_loadu_si128((const __m128i *)(p + 0)));
    x2 = _mm_xor_si128(_mm_xor_si128(x2, y2), _mm_loadu_si128((const __m128i *)(p + 16)));
    x3 = _mm_xor_si128(_mm_xor_si128(x3, y3), _mm_loadu_si128((const __m128i *)(p + 32)));
    x4 = _mm_xor_si128(_mm_xor_si128(x4, y4), _mm_loadu_si128((const __m128i *)(p + 48)));
    p += 64;
    n -= 64;
  }
#define FOLD1(acc, nxt)                                             \
  do {                                                              \
    __m128i hi_ = _mm_clmulepi64_si128(acc, r4r3, 0x11);           \
    acc = _mm_clmulepi64_si128(acc, r4r3, 0x00);                    \
    acc = _mm_xor_si128(_mm_xor_si128(acc, hi_), nxt);              \
  } while (0)
  FOLD1(x1, x2);
  FOLD1(x1, x3);
  FOLD1(x1, x4);
  while (n >= 16) {
    FOLD1(x1, _mm_loadu_si128((const __m128i *)p));
    p += 16;
    n -= 16;
  }
#undef FOLD1
  /* 128 -> 64 bits (also appends 32 zero bits) */
  __m128i t = _mm_clmulepi64_si128(r4r3, x1, 0x01);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), t);
  /* 64 -> 32 fold */
  t = _mm_and_si128(x1, mask32);
  x1 = _mm_srli_si128(x1, 4);
  t = _mm_clmulepi64_si128(t, r5, 0x00);
  x1 = _mm_xor_si128(x1, t);
  /* Barrett reduction */
  t = _mm_and_si128(x1, mask32);
  t = _mm_clmulepi64_si128(t, rupoly, 0x10);
  t = _mm_and_si128(t, mask32);
  t = _mm_clmulepi64_si128(t, rupoly, 0x00);
  x1 = _mm_xor_si128(x1, t);
  return (uint32_t)_mm_extract_epi32(x1, 1);
}
#endif

/* Go archUpdateIEEE (crc32_amd64.go): CLMUL on the 16-aligned prefix of
 * inputs >= 64 bytes, slicing-by-8 on the remainder. */
uint32_t oc_crc32_go_amd64(uint32_t crc, const uint8_t *p, size_t n) {
#if defined(__x86_64__)
  static int have = -1;
  if (have < 0) have = oc_have_pclmul();
  if (have && n >= 64) {
    size_t left = n & 15, todo = n - left;
    crc = ~clmul_fold(~crc, p, todo);
    p += todo;
    n = left;
  }
  if (n == 0) return crc;
#endif
  return oc_crc32_slicing8(crc, p, n);
}

uint32_t oc_checksum_ieee(const uint8_t *p, size_t n) { return oc_crc32_go_amd64(0, p, n); }

/* ------------------------------------------------------------------------ */
/* utils/crc/crc_util.go                                                    */
const char *oc_strerror(int code) {
  switch (code) {
    case OC_OK: return "";
    case OC_ERR_INVALID_BLOCK: return "invalid block data";                           /* :90 */
    case OC_ERR_CRC_MISMATCH: return "CRC mismatch in block";                         /* :96 */
    case OC_ERR_TOO_SHORT: return "data is too short to contain a complete block";    /* :108 */
    case OC_ERR_WAL_FRAGMENT_TYPE: return "unknown fragment type";                    /* wal.go:451 */
    case OC_ERR_WAL_TRUNCATED: return "WAL fragment overruns its block";             /* Go panics */
    default: return "unknown error";
  }
}

/* GetCRC, crc_util.go:15-17 */
uint32_t oc_get_crc(const uint8_t *p, size_t n) { return oc_checksum_ieee(p, n); }

/* AddCRCToBlockData, crc_util.go:21-33: in place, len<4 untouched */
void oc_add_crc_to_block_data(uint8_t *p, size_t n) {
  if (n < OC_CRC_SIZE) return;
  uint32_t c = oc_get_crc(p + OC_CRC_SIZE, n - OC_CRC_SIZE);
  memcpy(p, &c, 4); /* binary.LittleEndian.PutUint32 (host is little-endian) */
}

/* AddCRCsToData, crc_util.go:41-64: 4092-byte payload chunks into zeroed
 * 4096-byte blocks; output length = ceil(n/4092)*4096 (0 for n==0). */
size_t oc_add_crcs_to_data(const uint8_t *src, size_t n, uint8_t *dst) {
  const size_t per = OC_BLOCK_SIZE - OC_CRC_SIZE;
  size_t out = 0;
  for (size_t i = 0; i < n; i += per) {
    uint8_t *blk = dst + out;
    size_t end = i + per;
    if (end > n) end = n;
    memset(blk, 0, OC_BLOCK_SIZE);
    memcpy(blk + OC_CRC_SIZE, src + i, end - i);
    oc_add_crc_to_block_data(blk, OC_BLOCK_SIZE);
    out += OC_BLOCK_SIZE;
  }
  return out;
}

/* SizeAfterAddingCRCs, crc_util.go:69-74: float64 ceil, int(), uint64 math */
uint64_t oc_size_after_adding_crcs(uint64_t n) {
  const double per = (double)(OC_BLOCK_SIZE - OC_CRC_SIZE);
  int64_t nb = (int64_t)ceil((double)n / per); /* < 2^63 for every uint64 n */
  return n + (uint64_t)nb * OC_CRC_SIZE;
}

/* SizeWithoutCRCs, crc_util.go:79-83: wraps for 0 < n < 4 */
uint64_t oc_size_without_crcs(uint64_t n) {
  uint64_t nb = (uint64_t)ceil((double)n / (double)OC_BLOCK_SIZE);
  return n - nb * OC_CRC_SIZE;
}

/* CheckBlockIntegrity, crc_util.go:88-100 */
int oc_check_block_integrity(const uint8_t *p, size_t n) {
  if (n < OC_CRC_SIZE) return OC_ERR_INVALID_BLOCK;
  uint32_t stored = le32(p);
  uint32_t computed = oc_checksum_ieee(p + OC_CRC_SIZE, n - OC_CRC_SIZE);
  return stored != computed ? OC_ERR_CRC_MISMATCH : OC_OK;
}

/* FixLastBlockCRC, crc_util.go:106-122 (the :112-114 branch is unreachable) */
int oc_fix_last_block_crc(uint8_t *p, size_t n) {
  if (n < OC_BLOCK_SIZE) return OC_ERR_TOO_SHORT;
  size_t complete = n / OC_BLOCK_SIZE;
  oc_add_crc_to_block_data(p + (complete - 1) * OC_BLOCK_SIZE, OC_BLOCK_SIZE);
  return OC_OK;
}

/* BlockManager.ReadFromDisk, lsm/block_manager/block_manager.go:189-242, over
 * an in-memory image: `blocks` holds the blocks from index start_offset /
 * block_size on; `avail` bytes of it exist, the rest reads as zeros (the
 * short-read / EOF behaviour of readBlockFromDisk, :130-146).  Each touched
 * block is checked with CheckBlockIntegrity over the whole block (:215) before
 * its bytes are appended.  On error *bad_block = relative index of the block. */
int oc_read_from_disk(const uint8_t *blocks, uint64_t avail, uint32_t block_size, uint64_t start_offset,
                      uint64_t size, uint8_t *out, uint64_t *final_offset, int64_t *bad_block) {
  const uint64_t B = block_size;
  uint64_t block_offset = start_offset % B;
  if (block_offset < OC_CRC_SIZE) block_offset = OC_CRC_SIZE; /* :198-201 */
  uint8_t *blk = (uint8_t *)malloc(B);
  uint64_t cur = 0, remaining = size, produced = 0;
  *bad_block = -1;
  while (remaining > 0) {
    /* ReadBlock: make([]byte, blockSize) + file.Read (zeros past EOF) */
    memset(blk, 0, B);
    const uint64_t o = cur * B;
    if (o < avail) memcpy(blk, blocks + o, (avail - o) < B ? (avail - o) : B);
    int rc = oc_check_block_integrity(blk, B); /* :215 */
    if (rc != OC_OK) {
      *bad_block = (int64_t)cur;
      free(blk);
      return rc;
    }
    uint64_t take = B - block_offset; /* :221-225 */
    if (take > remaining) take = remaining;
    memcpy(out + produced, blk + block_offset, take);
    produced += take;
    remaining -= take;
    cur++;
    block_offset = OC_CRC_SIZE;
  }
  free(blk);
  /* :237-239 */
  *final_offset = oc_size_after_adding_crcs(oc_size_without_crcs(start_offset) + size);
  return OC_OK;
}

/* ------------------------------------------------------------------------ */
/* Threaded batches (cpu_baseline and test checker)                         */
typedef struct {
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride;
  uint32_t ulen;
  uint32_t *out;
  size_t n;
  size_t *next; /* shared work counter: threads take OC_CHUNK items at a time */
  int skip;     /* 4 = block mode (CRC of blk[4:]), 0 = whole message */
} job_t;

/* Dynamic chunks rather than one static range per thread: on a shared host a
 * thread that loses its CPU for a while no longer holds up the whole batch
 * (the cpu_baseline's 16-thread spread was +-25 % with static ranges). */
#define OC_CHUNK 64

static void *run_job(void *arg) {
  job_t *j = (job_t *)arg;
  for (;;) {
    size_t lo = __atomic_fetch_add(j->next, OC_CHUNK, __ATOMIC_RELAXED);
    if (lo >= j->n) break;
    size_t hi = lo + OC_CHUNK < j->n ? lo + OC_CHUNK : j->n;
    for (size_t i = lo; i < hi; i++) {
      uint64_t o = j->off ? j->off[i] : (uint64_t)i * j->stride;
      uint32_t l = j->len ? j->len[i] : j->ulen;
      if (j->skip && l < (uint32_t)j->skip) {
        j->out[i] = 0;
        continue;
      }
      j->out[i] = oc_checksum_ieee(j->base + o + j->skip, l - j->skip);
    }
  }
  return NULL;
}

static void run_batch(job_t proto, size_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
  pthread_t th[256];
  size_t next = 0;
  proto.n = n;
  proto.next = &next;
  if (nthreads == 1) {
    run_job(&proto);
    return;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &proto);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void oc_crc32_blocks(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint64_t stride, uint32_t ulen, uint32_t *out, size_t nblocks,
                     int nthreads) {
  job_t p = {base, off, len, stride, ulen, out, 0, NULL, 4};
  run_batch(p, nblocks, nthreads);
}

void oc_crc32_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       uint32_t *out, size_t n, int nthreads) {
  job_t p = {base, off, len, 0, 0, out, 0, NULL, 0};
  run_batch(p, n, nthreads);
}

/* ------------------------------------------------------------------------ */
/* Synthetic inputs: splitmix64 finaliser over a (seed, block, word) counter */
uint64_t oc_splitmix64(uint64_t seed, uint64_t block, uint64_t word) {
  uint64_t z = seed + ((block << 21) + word) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oc_fill_block(uint64_t seed, uint64_t block, uint8_t *dst, size_t len) {
  for (size_t w = 0; w < len / 8; w++) {
    uint64_t v = oc_splitmix64(seed, block, w);
    memcpy(dst + 8 * w, &v, 8);
  }
}

/* Blocks first .. first+n-1 of a uniform batch (block_bytes each) into dst,
 * on nthreads threads: the host copy of what hc_dev_fill_range writes, for
 * full-size checks that regenerate a batch by index instead of copying it
 * back from the device. */
typedef struct {
  uint64_t seed, first, n, bytes;
  uint8_t *dst;
  size_t *next;
} fill_job_t;

static void *run_fill(void *arg) {
  fill_job_t *j = (fill_job_t *)arg;
  for (;;) {
    size_t lo = __atomic_fetch_add(j->next, OC_CHUNK, __ATOMIC_RELAXED);
    if (lo >= j->n) break;
    size_t hi = lo + OC_CHUNK < j->n ? lo + OC_CHUNK : j->n;
    for (size_t i = lo; i < hi; i++) oc_fill_block(j->seed, j->first + i, j->dst + i * j->bytes, j->bytes);
  }
  return NULL;
}

void oc_fill_blocks_mt(uint64_t seed, uint64_t first, uint64_t n, uint64_t block_bytes, uint8_t *dst, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  size_t next = 0;
  fill_job_t j = {seed, first, n, block_bytes, dst, &next};
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_fill, &j);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

uint32_t oc_mixed_size(uint64_t seed, uint64_t block) {
  /* word index 2^21-1 is never a data word of a <=16 MiB block */
  uint64_t r = oc_splitmix64(seed ^ 0x5A5A5A5A5A5A5A5Aull, block, (1u << 21) - 1);
  return 4096u << (uint32_t)(r % 3);
}

/* ------------------------------------------------------------------------ */
/* WAL framing, lsm/wal/wal.go:177-283                                      */
#define WAL_HDR 17 /* wal_header.go:16: size u64 | type u8 | log u64 */
enum { FRAG_FIRST = 1, FRAG_MIDDLE = 2, FRAG_LAST = 3, FRAG_FULL = 4 };

uint32_t oc_wal_record_size(uint64_t seed, uint64_t i, uint32_t lo, uint32_t hi) {
  /* integer log-uniform: uniform octave, uniform within the octave, clamped */
  uint64_t r = oc_splitmix64(seed ^ 0x3C3C3C3C3C3C3C3Cull, i, 0);
  uint32_t elo = 0, ehi = 0;
  while ((1u << (elo + 1)) <= lo) elo++;
  while ((1ull << ehi) < hi) ehi++;
  uint32_t e = elo + (uint32_t)(r % (ehi - elo));
  uint64_t s = (1ull << e) + ((r >> 8) % (1ull << e));
  if (s < lo) s = lo;
  if (s > hi) s = hi;
  return (uint32_t)s;
}

typedef struct {
  uint8_t *dst;
  uint64_t max_blocks, nblocks, blocks_in_log, log_index, log_size;
  uint32_t bs, off;
  uint8_t *cur; /* current block (points into dst or a scratch block) */
  int stamp, full;
  uint8_t scratch[65536]; /* must stay the last member (see oc_wal_frame) */
} walw_t;

static uint8_t *wal_block_ptr(walw_t *w) {
  if (w->dst && w->nblocks < w->max_blocks) return w->dst + w->nblocks * (uint64_t)w->bs;
  return w->scratch;
}
/* makeNewBlock, wal.go:273-283 */
static void wal_make_new_block(walw_t *w) {
  w->cur = wal_block_ptr(w);
  memset(w->cur, 0, w->bs);
  w->off = OC_CRC_SIZE;
  if (w->blocks_in_log >= w->log_size) {
    w->log_index++;
    w->blocks_in_log = 0;
  }
}
/* flushBlock, wal.go:260-271 */
static void wal_flush(walw_t *w) {
  if (w->stamp) oc_add_crc_to_block_data(w->cur, w->bs);
  w->nblocks++;
  w->blocks_in_log++;
  if (w->nblocks >= w->max_blocks) w->full = 1;
}
/* writeToBlock, wal.go:229-257 */
static int wal_write_to_block(walw_t *w, uint64_t seed, uint64_t rec, uint64_t pay_off,
                              uint32_t len, uint32_t total_len, uint8_t type) {
  if (w->off + WAL_HDR + len > w->bs) return -1; /* "not enough space in block" */
  uint8_t *h = w->cur + w->off;
  uint64_t sz = len, lg = w->log_index;
  memcpy(h, &sz, 8);
  h[8] = type;
  memcpy(h + 9, &lg, 8);
  /* serialized record bytes (record.go:107-119): ts8|tomb1|klen8|vlen8|key|value */
  uint8_t *d = h + WAL_HDR;
  const uint64_t ksz = total_len - 25 < 16 ? total_len - 25 : 16; /* records are >= 25 B */
  for (uint32_t k = 0; k < len; k++) {
    uint64_t pos = pay_off + k;
    uint8_t b;
    if (pos < 8) b = (uint8_t)(rec >> (8 * pos));                          /* timestamp */
    else if (pos == 8) b = 0;                                              /* tombstone */
    else if (pos < 17) b = (uint8_t)(ksz >> (8 * (pos - 9)));              /* key size */
    else if (pos < 25) b = (uint8_t)((total_len - 25 - ksz) >> (8 * (pos - 17))); /* value size */
    else b = (uint8_t)(oc_splitmix64(seed, rec, (pos - 25) >> 3) >> (8 * ((pos - 25) & 7)));
    d[k] = b;
  }
  w->off += WAL_HDR + len;
  if (w->off == w->bs) {
    wal_flush(w);
    wal_make_new_block(w);
  }
  return 0;
}

uint64_t oc_wal_frame(uint64_t seed, const uint32_t *rec_sizes, uint64_t nrec, uint32_t bs,
                      uint8_t *dst, uint64_t max_blocks, int stamp, oc_wal_stats *st,
                      uint64_t *next_rec) {
  static __thread walw_t w; /* scratch is large; keep off the stack */
  memset(&w, 0, sizeof(w) - sizeof(w.scratch));
  w.dst = dst;
  w.max_blocks = max_blocks;
  w.bs = bs;
  w.stamp = stamp;
  w.log_index = 1;
  w.log_size = 16; /* config.go default WAL.LogSize */
  oc_wal_stats s = {0, 0, 0, 0};
  wal_make_new_block(&w);
  uint64_t r = 0;
  for (; r < nrec && !w.full; r++) {
    uint32_t S = rec_sizes[r];
    uint32_t need = WAL_HDR + S;
    if (bs - w.off < need) { /* wal.go:182 */
      wal_flush(&w);
      wal_make_new_block(&w);
      if (w.full) break;
      if (need > bs) { /* writeFragmentedRecord, wal.go:199-225 */
        uint32_t maxp = bs - WAL_HDR - OC_CRC_SIZE;
        uint32_t nf = (uint32_t)ceil((double)S / (double)maxp);
        uint32_t po = 0;
        for (uint32_t i = 0; i < nf && !w.full; i++) {
          uint32_t fl = S - po < maxp ? S - po : maxp;
          uint8_t t = FRAG_MIDDLE;
          if (i == 0) t = FRAG_FIRST;
          else if (i == nf - 1) t = FRAG_LAST;
          wal_write_to_block(&w, seed, r, po, fl, S, t);
          po += fl;
          s.fragments++;
        }
        s.records++;
        continue;
      }
    }
    if (wal_write_to_block(&w, seed, r, 0, S, S, FRAG_FULL) != 0) {
      s.refused++; /* 4092 < 17+S <= 4096 (for bs=4096): wal.go:238-240 */
      continue;
    }
    s.records++;
  }
  if (!w.full) wal_flush(&w); /* Close(), wal.go:286+ */
  s.blocks = w.nblocks;
  if (st) *st = s;
  if (next_rec) *next_rec = r;
  return w.nblocks;
}

/* ------------------------------------------------------------------------ */
/* WAL recovery, lsm/wal/wal.go:362-455 (recoverMemtable +                  */
/* processBlockForRecovery) over a run of written blocks.  One call = one    */
/* memtable: the fragment buffer is local (:365), max_records plays         */
/* memtable.IsFull (0 = never full).  Records are the payload bytes          */
/* record.Deserialize would receive, appended to rec_buf in order.          */
int oc_wal_replay(const uint8_t *blocks, uint64_t nblocks, uint32_t bs, uint64_t start_block,
                  uint64_t start_offset, uint64_t max_records, uint8_t *rec_buf, uint64_t *rec_off,
                  uint64_t *rec_len, uint64_t *nrec, uint64_t *pos_block, uint64_t *pos_offset,
                  int64_t *bad_block) {
  uint8_t *frag = (uint8_t *)malloc((size_t)bs * (nblocks + 1));
  uint64_t flen = 0, used = 0, n = 0;
  uint64_t blk = start_block, off = start_offset;
  int rc = OC_OK, full = 0;
  *bad_block = -1;
  for (; blk < nblocks && !full; blk++, off = OC_CRC_SIZE) { /* :370-396 */
    const uint8_t *b = blocks + blk * (uint64_t)bs;
    if (oc_check_block_integrity(b, bs) != OC_OK) { /* :383-386 */
      rc = OC_ERR_CRC_MISMATCH;
      *bad_block = (int64_t)blk;
      break;
    }
    while (off < bs) { /* processBlockForRecovery, :412-453 */
      uint64_t z = off;
      while (z < bs && b[z] == 0) z++;
      if (z == bs) { /* rest of the block is padding (:415-419) */
        flen = 0;
        break;
      }
      if (off + 17 > bs) { rc = OC_ERR_WAL_TRUNCATED; break; } /* nil header in Go */
      uint64_t size;
      memcpy(&size, b + off, 8);
      const uint8_t type = b[off + 8];
      off += 17;
      if (size > bs - off) { rc = OC_ERR_WAL_TRUNCATED; break; } /* slice bounds panic in Go */
      const uint8_t *pay = b + off;
      off += size;
      if (type == 4) { /* FRAGMENT_FULL */
        memcpy(rec_buf + used, pay, size);
        rec_off[n] = used;
        rec_len[n] = size;
        used += size;
        n++;
        if (max_records && n >= max_records) { full = 1; break; }
      } else if (type == 1 || type == 2) { /* FIRST, MIDDLE */
        memcpy(frag + flen, pay, size);
        flen += size;
      } else if (type == 3) { /* LAST */
        memcpy(frag + flen, pay, size);
        flen += size;
        memcpy(rec_buf + used, frag, flen);
        rec_off[n] = used;
        rec_len[n] = flen;
        used += flen;
        n++;
        flen = 0;
        if (max_records && n >= max_records) { full = 1; break; }
      } else {
        rc = OC_ERR_WAL_FRAGMENT_TYPE;
        break;
      }
    }
    if (rc != OC_OK) break;
  }
  free(frag);
  *nrec = n;
  if (rc == OC_OK) { /* :392-393: the next memtable starts at the next block */
    *pos_block = blk;
    *pos_offset = OC_CRC_SIZE;
  } else {
    *pos_block = blk;
    *pos_offset = off;
  }
  return rc;
}

