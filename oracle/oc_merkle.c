/*
 * oc_merkle.c — CPU oracle for row f4's Merkle/MD5 integrity check.
 *
 * TEST INFRASTRUCTURE ONLY (see hc_oracle.h).  Restates:
 *   - MD5 (RFC 1321), the algorithm of Go's crypto/md5 (go 1.23.2 stdlib, not
 *     vendored under /root/reference), as md5.Sum is called by
 *     lsm/sstable/sstable.go:2358 (record leaves) and by
 *     lsm/sstable/merkle_tree/merkle_tree.go:37,48,50,74 (empty tree, leaves,
 *     parent nodes);
 *   - merkle_tree.go: NewMerkleTree (:36-81, hashedAlready = true as
 *     CheckIntegrity calls it at sstable.go:2368), Serialize (:173-187, DFS
 *     pre-order), Deserialize/DeserializeDFS (:192-226) and Validate/DeepValidate
 *     (:115-147), with pointer-built nodes exactly as Go builds them.
 * Pinned by the RFC 1321 test suite, Python hashlib.md5 vectors and the
 * expected roots of merkle_tree_test.go:11-21 (tests/golden/).
 */
#include <stdlib.h>
#include <string.h>

#include "hc_oracle.h"

/* ---- MD5 (RFC 1321 section 3.4, reference implementation structure) ---- */
static const uint32_t T[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                          5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                          4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                          6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static uint32_t rotl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

static void md5_block(uint32_t st[4], const uint8_t *b) {
  uint32_t X[16];
  for (int i = 0; i < 16; i++)
    X[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
  uint32_t a = st[0], bb = st[1], c = st[2], d = st[3];
  for (int i = 0; i < 64; i++) {
    uint32_t f;
    int k;
    if (i < 16) {
      f = (bb & c) | (~bb & d);
      k = i;
    } else if (i < 32) {
      f = (bb & d) | (c & ~d);
      k = (5 * i + 1) & 15;
    } else if (i < 48) {
      f = bb ^ c ^ d;
      k = (3 * i + 5) & 15;
    } else {
      f = c ^ (bb | ~d);
      k = (7 * i) & 15;
    }
    const uint32_t t = d;
    d = c;
    c = bb;
    bb = bb + rotl(a + f + T[i] + X[k], S[i]);
    a = t;
  }
  st[0] += a;
  st[1] += bb;
  st[2] += c;
  st[3] += d;
}

void oc_md5(const uint8_t *p, size_t n, uint8_t out[16]) {
  uint32_t st[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
  size_t i = 0;
  for (; i + 64 <= n; i += 64) md5_block(st, p + i);
  /* padding: 0x80, zeros to 56 mod 64, then the bit length (little endian) */
  uint8_t tail[128];
  const size_t r = n - i;
  memset(tail, 0, sizeof tail);
  if (r) memcpy(tail, p + i, r);
  tail[r] = 0x80;
  const size_t tl = r < 56 ? 64 : 128;
  const uint64_t bits = (uint64_t)n * 8;
  for (int k = 0; k < 8; k++) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
  md5_block(st, tail);
  if (tl == 128) md5_block(st, tail + 64);
  for (int k = 0; k < 4; k++)
    for (int j = 0; j < 4; j++) out[4 * k + j] = (uint8_t)(st[k] >> (8 * j));
}

void oc_md5_messages(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint8_t *out, size_t n) {
  for (size_t i = 0; i < n; i++) oc_md5(base + off[i], len[i], out + 16 * i);
}

/* ---- merkle_tree.go ------------------------------------------------------ */
typedef struct MNode {
  uint8_t h[16];
  struct MNode *l, *r;
} MNode;

typedef struct {  /* every node of one tree, for freeing */
  MNode **v;
  size_t n, cap;
} Arena;

static MNode *node_new(Arena *A, const uint8_t h[16]) {
  MNode *x = (MNode *)calloc(1, sizeof(MNode));
  if (h) memcpy(x->h, h, 16);
  if (A->n == A->cap) {
    A->cap = A->cap ? 2 * A->cap : 64;
    A->v = (MNode **)realloc(A->v, A->cap * sizeof(MNode *));
  }
  A->v[A->n++] = x;
  return x;
}

static void arena_free(Arena *A) {
  for (size_t i = 0; i < A->n; i++) free(A->v[i]);
  free(A->v);
  A->v = NULL;
  A->n = A->cap = 0;
}

/* NewMerkleTree(blocks, hashedAlready=true) (:36-81) */
static MNode *build(Arena *A, const uint8_t *leaves, uint64_t n) {
  if (n == 0) {
    uint8_t e[16];
    oc_md5(NULL, 0, e);
    return node_new(A, e);
  }
  MNode **nodes = (MNode **)malloc((n + 1) * sizeof(MNode *));
  uint64_t cnt = n;
  for (uint64_t i = 0; i < n; i++) nodes[i] = node_new(A, leaves + 16 * i);
  while (cnt > 1) {
    if (cnt % 2 == 1) nodes[cnt++] = node_new(A, NULL); /* neutral node: zero hash, no children */
    uint64_t m = 0;
    for (uint64_t i = 0; i < cnt; i += 2) {
      uint8_t comb[32];
      memcpy(comb, nodes[i]->h, 16);
      memcpy(comb + 16, nodes[i + 1]->h, 16);
      uint8_t h[16];
      oc_md5(comb, 32, h);
      MNode *p = node_new(A, h);
      p->l = nodes[i];
      p->r = nodes[i + 1];
      nodes[m++] = p;
    }
    cnt = m;
  }
  MNode *root = nodes[0];
  free(nodes);
  return root;
}

/* Serialize (:173-187): DFS pre-order, 16 bytes per node */
static void ser(const MNode *x, uint8_t *out, uint64_t *pos) {
  if (out) memcpy(out + 16 * *pos, x->h, 16);
  (*pos)++;
  if (x->l) ser(x->l, out, pos);
  if (x->r) ser(x->r, out, pos);
}

/* DeserializeDFS (:229-250): every node takes children while bytes remain.
 * Go's recursion is unrolled here (a stored tree of 10^6 nodes would overflow
 * a C stack): a call that reads a node returns only once the bytes are
 * exhausted (its left call does, by induction), so the `*offset < len(data)`
 * test before the right child is always false -- every node gets the next
 * node as its left child and no right child. */
static MNode *deser(Arena *A, const uint8_t *d, uint64_t len, uint64_t *off) {
  MNode *root = NULL, *prev = NULL;
  while (*off < len) {
    uint8_t h[16] = {0};
    memcpy(h, d + *off, len - *off >= 16 ? 16 : len - *off); /* copy(hash[:], data[off:off+16]) */
    *off += 16;
    MNode *x = node_new(A, h);
    if (prev)
      prev->l = x;
    else
      root = x;
    prev = x;
  }
  return root;
}

typedef struct {
  uint8_t *m1, *m2;
  uint64_t cap, n;
} Mism;

static const uint8_t ZERO16[16];

/* DeepValidate (:129-147) */
static void deep(const MNode *a, const MNode *b, Mism *M) {
  if (!a || !b) return;
  if (memcmp(a->h, b->h, 16) == 0) return;
  if (!a->l && !a->r && !b->l && !b->r) {
    if (M->n < M->cap) {
      if (M->m1) memcpy(M->m1 + 16 * M->n, a->h, 16);
      if (M->m2) memcpy(M->m2 + 16 * M->n, b->h, 16);
    }
    M->n++;
  } else if (memcmp(a->h, ZERO16, 16) != 0 || memcmp(b->h, ZERO16, 16) != 0) {
    deep(a->l, b->l, M);
    deep(a->r, b->r, M);
  }
}

void oc_merkle_root(const uint8_t *leaves, uint64_t n, uint8_t root[16]) {
  Arena A = {0};
  memcpy(root, build(&A, leaves, n)->h, 16);
  arena_free(&A);
}

uint64_t oc_merkle_serialize(const uint8_t *leaves, uint64_t n, uint8_t *out) {
  Arena A = {0};
  uint64_t pos = 0;
  ser(build(&A, leaves, n), out, &pos);
  arena_free(&A);
  return 16 * pos;
}

int oc_merkle_validate(const uint8_t *leaves, uint64_t n, const uint8_t *stored, uint64_t stored_len,
                       uint8_t *mism1, uint8_t *mism2, uint64_t cap, uint64_t *nmism) {
  Arena A = {0};
  const MNode *t1 = build(&A, leaves, n);
  uint64_t off = 0;
  const MNode *t2 = deser(&A, stored, stored_len, &off);
  *nmism = 0;
  if (!t2) { /* Deserialize of no bytes: a nil root, Go's Validate panics */
    arena_free(&A);
    return -1;
  }
  int valid = memcmp(t1->h, t2->h, 16) == 0;
  if (!valid) {
    Mism M = {mism1, mism2, cap, 0};
    deep(t1, t2, &M);
    *nmism = M.n;
  }
  arena_free(&A);
  return valid;
}

/* tree(leaves1).Validate(tree(leaves2)) for two built trees (merkle_tree_test.go:127-180) */
int oc_merkle_validate_trees(const uint8_t *l1, uint64_t n1, const uint8_t *l2, uint64_t n2, uint8_t *mism1,
                             uint8_t *mism2, uint64_t cap, uint64_t *nmism) {
  Arena A = {0};
  const MNode *t1 = build(&A, l1, n1), *t2 = build(&A, l2, n2);
  *nmism = 0;
  int valid = memcmp(t1->h, t2->h, 16) == 0;
  if (!valid) {
    Mism M = {mism1, mism2, cap, 0};
    deep(t1, t2, &M);
    *nmism = M.n;
  }
  arena_free(&A);
  return valid;
}
