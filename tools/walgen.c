/*
 * walgen.c — parallel generator of HundDB WAL images for the config-5
 * benchmark (10M records, 64 B..64 KiB, framed into 4 KiB WAL blocks).
 *
 * Benchmark infrastructure, not product and not the oracle.  It reproduces the
 * framing of /root/reference/lsm/wal/wal.go:177-283 (WriteRecord,
 * writeFragmentedRecord, writeToBlock, flushBlock, makeNewBlock, Close) and the
 * header of wal_header.go:5-77 in two phases so it can run on many threads:
 *   wg_plan    sequential: where every record / fragment lands (cheap, sizes only)
 *   wg_render  parallel over block ranges: write headers + payload bytes and
 *              stamp each block's CRC (flushBlock's AddCRCToBlockData).
 * tests/test_walgen.py checks its output byte-for-byte against the oracle's
 * sequential restatement (oracle/hc_oracle.c oc_wal_frame).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define HDR 17
#define CRC_SIZE 4
#define NONE 0xFFFFFFFFu
enum { KIND_FULL = 0, KIND_FRAG = 1, KIND_REFUSED = 2 };

static uint32_t T8[8][256];
static pthread_once_t once = PTHREAD_ONCE_INIT;
static void init_tab(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    T8[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++)
    for (int t = 1; t < 8; t++) T8[t][i] = (T8[t - 1][i] >> 8) ^ T8[0][T8[t - 1][i] & 0xFF];
}
static uint32_t crc32_ieee(const uint8_t *p, size_t n) {
  uint32_t c = ~0u;
  while (n >= 8) {
    uint32_t a, b;
    memcpy(&a, p, 4);
    memcpy(&b, p + 4, 4);
    a ^= c;
    c = T8[7][a & 255] ^ T8[6][(a >> 8) & 255] ^ T8[5][(a >> 16) & 255] ^ T8[4][a >> 24] ^
        T8[3][b & 255] ^ T8[2][(b >> 8) & 255] ^ T8[1][(b >> 16) & 255] ^ T8[0][b >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ T8[0][(c ^ *p++) & 255];
  return ~c;
}

static inline uint64_t splitmix(uint64_t seed, uint64_t blk, uint64_t w) {
  uint64_t z = seed + ((blk << 21) + w) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Integer log-uniform record size (same draw as oc_wal_record_size). */
uint32_t wg_record_size(uint64_t seed, uint64_t i, uint32_t lo, uint32_t hi) {
  uint64_t r = splitmix(seed ^ 0x3C3C3C3C3C3C3C3Cull, i, 0);
  uint32_t elo = 0, ehi = 0;
  while ((1u << (elo + 1)) <= lo) elo++;
  while ((1ull << ehi) < hi) ehi++;
  uint32_t e = elo + (uint32_t)(r % (ehi - elo));
  uint64_t s = (1ull << e) + ((r >> 8) % (1ull << e));
  if (s < lo) s = lo;
  if (s > hi) s = hi;
  return (uint32_t)s;
}

void wg_record_sizes(uint64_t seed, uint64_t n, uint32_t lo, uint32_t hi, uint32_t *out) {
  for (uint64_t i = 0; i < n; i++) out[i] = wg_record_size(seed, i, lo, hi);
}

/* Plan.  rec_block/rec_off/rec_kind: where record r's first header goes.
 * first_rec[b]: first record writing into block b (NONE = empty block).
 * Returns the number of blocks (Close() flushes the open block); *refused
 * counts records writeToBlock rejects (4092 < 17+S <= 4096 for bs=4096). */
uint64_t wg_plan(const uint32_t *size, uint64_t nrec, uint32_t bs, uint32_t *rec_block,
                 uint16_t *rec_off, uint8_t *rec_kind, uint32_t *first_rec, uint64_t max_blocks,
                 uint64_t *refused) {
  uint64_t blk = 0, nref = 0;
  uint32_t off = CRC_SIZE;
  const uint32_t maxp = bs - HDR - CRC_SIZE; /* wal.go:200 */
#define TOUCH(b, r)                                    \
  do {                                                 \
    if ((b) < max_blocks && first_rec[b] == NONE) first_rec[b] = (uint32_t)(r); \
  } while (0)
  for (uint64_t b = 0; b < max_blocks; b++) first_rec[b] = NONE;
  for (uint64_t r = 0; r < nrec; r++) {
    const uint32_t S = size[r], need = HDR + S;
    if (bs - off < need) { /* wal.go:182-192: flush, new block, maybe fragment */
      blk++;
      off = CRC_SIZE;
      if (need > bs) {
        const uint32_t nf = (S + maxp - 1) / maxp;
        rec_block[r] = (uint32_t)blk;
        rec_off[r] = CRC_SIZE;
        rec_kind[r] = KIND_FRAG;
        for (uint32_t i = 0; i < nf; i++) TOUCH(blk + i, r);
        const uint32_t last = S - (nf - 1) * maxp;
        blk += nf - 1;
        off = CRC_SIZE + HDR + last;
        if (off == bs) { /* exactly full -> flushed + new block */
          blk++;
          off = CRC_SIZE;
        }
        continue;
      }
    }
    if (off + need > bs) { /* writeToBlock: "not enough space in block" */
      rec_block[r] = (uint32_t)blk;
      rec_off[r] = (uint16_t)off;
      rec_kind[r] = KIND_REFUSED;
      nref++;
      continue;
    }
    rec_block[r] = (uint32_t)blk;
    rec_off[r] = (uint16_t)off;
    rec_kind[r] = KIND_FULL;
    TOUCH(blk, r);
    off += need;
    if (off == bs) {
      blk++;
      off = CRC_SIZE;
    }
  }
#undef TOUCH
  if (refused) *refused = nref;
  return blk + 1; /* Close() flushes the open block */
}

static void put_payload(uint8_t *d, uint64_t seed, uint64_t rec, uint32_t total, uint32_t pos,
                        uint32_t n) {
  const uint64_t ksz = total - 25 < 16 ? total - 25 : 16;
  uint32_t k = 0;
  for (; k < n && pos + k < 25; k++) {
    const uint32_t p = pos + k;
    uint8_t b;
    if (p < 8) b = (uint8_t)(rec >> (8 * p));
    else if (p == 8) b = 0;
    else if (p < 17) b = (uint8_t)(ksz >> (8 * (p - 9)));
    else b = (uint8_t)((total - 25 - ksz) >> (8 * (p - 17)));
    d[k] = b;
  }
  while (k < n) {
    const uint32_t q = pos + k - 25;
    const uint64_t w = splitmix(seed, rec, q >> 3);
    const uint32_t sh = q & 7;
    if (sh == 0 && n - k >= 8) {
      memcpy(d + k, &w, 8);
      k += 8;
    } else {
      d[k++] = (uint8_t)(w >> (8 * sh));
    }
  }
}

static void put_header(uint8_t *h, uint64_t size, uint8_t type, uint64_t log) {
  memcpy(h, &size, 8); /* wal_header.go:57-63, little-endian */
  h[8] = type;
  memcpy(h + 9, &log, 8);
}

typedef struct {
  uint64_t seed;
  const uint32_t *size;
  uint64_t nrec;
  uint32_t bs;
  const uint32_t *rec_block;
  const uint16_t *rec_off;
  const uint8_t *rec_kind;
  const uint32_t *first_rec;
  uint64_t b0, b1; /* global block range of this job */
  uint8_t *dst;    /* receives blocks b0..b1 */
  int stamp;
} job_t;

static void render_range(const job_t *j) {
  const uint32_t bs = j->bs, maxp = bs - HDR - CRC_SIZE;
  for (uint64_t b = j->b0; b < j->b1; b++) {
    uint8_t *blk = j->dst + (b - j->b0) * (uint64_t)bs;
    memset(blk, 0, bs);
    const uint64_t log = 1 + b / 16; /* makeNewBlock rolls every LOG_SIZE=16 blocks */
    uint32_t r = j->first_rec[b];
    for (; r != NONE && r < j->nrec && j->rec_block[r] <= b; r++) {
      const uint32_t S = j->size[r];
      if (j->rec_kind[r] == KIND_REFUSED) continue;
      if (j->rec_kind[r] == KIND_FULL) {
        if (j->rec_block[r] != b) continue;
        uint8_t *h = blk + j->rec_off[r];
        put_header(h, S, 4, log);
        put_payload(h + HDR, j->seed, r, S, 0, S);
      } else {
        const uint32_t nf = (S + maxp - 1) / maxp;
        if (b >= j->rec_block[r] + (uint64_t)nf) continue;
        const uint32_t i = (uint32_t)(b - j->rec_block[r]);
        const uint32_t fl = i + 1 < nf ? maxp : S - (nf - 1) * maxp;
        const uint8_t type = i == 0 ? 1 : (i == nf - 1 ? 3 : 2);
        put_header(blk + CRC_SIZE, fl, type, log);
        put_payload(blk + CRC_SIZE + HDR, j->seed, r, S, i * maxp, fl);
      }
    }
    if (j->stamp) {
      const uint32_t c = crc32_ieee(blk + CRC_SIZE, bs - CRC_SIZE);
      memcpy(blk, &c, 4);
    }
  }
}

static void *run(void *a) {
  render_range((const job_t *)a);
  return NULL;
}

/* Render blocks [b0, b1) into dst on `threads` threads. */
void wg_render(uint64_t seed, const uint32_t *size, uint64_t nrec, uint32_t bs, const uint32_t *rec_block,
               const uint16_t *rec_off, const uint8_t *rec_kind, const uint32_t *first_rec, uint64_t b0,
               uint64_t b1, uint8_t *dst, int stamp, int threads) {
  pthread_once(&once, init_tab);
  if (threads < 1) threads = 1;
  if (threads > 128) threads = 128;
  job_t jobs[128];
  pthread_t th[128];
  const uint64_t n = b1 - b0;
  for (int t = 0; t < threads; t++) {
    job_t j = {seed, size, nrec, bs, rec_block, rec_off, rec_kind, first_rec,
               b0 + n * t / threads, b0 + n * (t + 1) / threads, NULL, stamp};
    j.dst = dst + (j.b0 - b0) * (uint64_t)bs;
    jobs[t] = j;
  }
  for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, run, &jobs[t]);
  render_range(&jobs[0]);
  for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
}
