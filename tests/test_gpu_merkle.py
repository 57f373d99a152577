"""Row f4 on the GPU: md5.Sum leaves (k_md5) and Merkle levels
(k_merkle_level) through the C ABI vs the oracle (oracle/oc_merkle.c, pinned
to hashlib and merkle_tree_test.go's roots in test_merkle.py), bit-exact.

Edge cases: every tail length around the MD5 padding boundary (55/56/63/64,
119/120), empty records, unaligned record starts, uniform-stride batches,
odd level counts (zero padding nodes, merkle_tree.go:60-66), n = 0 / 1, and a
corrupted record found by CheckIntegrity's Validate (sstable.go:2405-2416).
"""
import hashlib

import numpy as np
import pytest

from hunddb_amd import merkle as M

pytestmark = pytest.mark.gpu


def _packed(rng, lens, pad=1):
    """Records back to back, starting at byte `pad` (unaligned)."""
    lens = np.asarray(lens, dtype=np.uint32)
    off = np.zeros(len(lens), dtype=np.uint64)
    if len(lens):
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    off += pad
    total = int(off[-1] + lens[-1]) if len(lens) else pad
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
    return buf, off, lens


def _oracle_md5(oracle, buf, off, lens):
    out = np.empty((len(off), 16), dtype=np.uint8)
    oracle.lib().oc_md5_messages(buf.ctypes.data, off.ctypes.data, lens.ctypes.data, out.ctypes.data, len(off))
    return out


def _dev_md5(torch, buf, off, lens):
    dbuf = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(len(off) * 16, dtype=torch.uint8, device="cuda")
    M.dev_md5_messages(dbuf, out, off=doff, lens=dlen, n=len(off))
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(-1, 16)


def test_md5_padding_boundaries(cuda, oracle):
    torch = cuda
    rng = np.random.default_rng(1)
    lens = [0, 1, 3, 4, 15, 16, 17, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129, 1000, 4092, 4096, 65536]
    lens = lens * 5  # several start alignments per length
    buf, off, ln = _packed(rng, lens, pad=3)
    got = _dev_md5(torch, buf, off, ln)
    for i in range(len(ln)):
        want = hashlib.md5(buf[int(off[i]):int(off[i]) + int(ln[i])].tobytes()).digest()
        assert got[i].tobytes() == want, (i, int(ln[i]), int(off[i]) % 16)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 1023, 1025])
def test_md5_small_batches(cuda, oracle, n):
    """Batches smaller than one wave's 64 lanes or one workgroup's range: idle
    waves and lanes, ragged last window; a 1 MiB record and empty records."""
    torch = cuda
    rng = np.random.default_rng(100 + n)
    lens = rng.integers(0, 5000, n).astype(np.uint32)
    lens[0] = 1 << 20
    if n > 2:
        lens[-1] = 0
    buf, off, ln = _packed(rng, lens, pad=7)
    got = _dev_md5(torch, buf, off, ln)
    want = _oracle_md5(oracle, buf, off, ln)
    assert (got == want).all()


def test_md5_records_batch_vs_oracle(cuda, oracle):
    """200k records, log-uniform 0 B .. 64 KiB (the record sizes of config 5),
    unaligned starts: every digest vs the oracle."""
    torch = cuda
    rng = np.random.default_rng(2)
    n = 200_000
    lens = np.minimum(np.exp(rng.uniform(0, np.log(65536), n)).astype(np.uint32), 65536)
    lens[rng.integers(0, n, 100)] = 0
    buf, off, ln = _packed(rng, lens, pad=5)
    got = _dev_md5(torch, buf, off, ln)
    want = _oracle_md5(oracle, buf, off, ln)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("case", ["skewed", "all_empty", "one_huge", "threshold"])
def test_md5_balanced_ranges(cuda, oracle, case):
    """From 16384 off/len messages k_md5's waves take ranges of equal work
    (k_md5_wsum / k_md5_split / k_md5_bounds): ranges of very unequal counts,
    all-equal weights, one wave's range a single 8 MiB record, and the
    threshold itself.  Every digest vs the oracle."""
    torch = cuda
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    if case == "skewed":
        lens = np.zeros(40_000, dtype=np.uint32)
        lens[20_000:] = rng.integers(0, 200, 20_000)
        lens[-300:] = 65536
    elif case == "all_empty":
        lens = np.zeros(50_000, dtype=np.uint32)
    elif case == "one_huge":
        lens = rng.integers(0, 3000, 40_000).astype(np.uint32)
        lens[12345] = 8 << 20
    else:
        lens = rng.integers(0, 9000, 16_384).astype(np.uint32)
    buf, off, ln = _packed(rng, lens, pad=3)
    got = _dev_md5(torch, buf, off, ln)
    want = _oracle_md5(oracle, buf, off, ln)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}"


def test_md5_uniform_stride(cuda, oracle, hc):
    torch = cuda
    n, size = 100_000, 4096
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(buf, 77, stride=size, ulen=size, nblocks=n)
    for ulen in (4096, 4092, 100):
        out = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        M.dev_md5_messages(buf, out, stride=size, ulen=ulen, n=n)
        torch.cuda.synchronize()
        host = buf.cpu().numpy()
        off = (np.arange(n, dtype=np.uint64) * size)
        lens = np.full(n, ulen, dtype=np.uint32)
        want = _oracle_md5(oracle, host, off, lens)
        assert (out.cpu().numpy().reshape(-1, 16) == want).all(), ulen


def test_host_records_larger_than_staging(cuda, oracle, hc):
    """Records over the 64 MiB staging slot (md5.Sum / GetCRC take any size):
    hashed on their own between ordinary records, host memory."""
    rng = np.random.default_rng(9)
    lens = np.array([100, (80 << 20) + 13, 5000, 70 << 20, 0, 333], np.uint32)
    buf, off, ln = _packed(rng, lens, pad=1)
    got = M.md5_records(buf, off, ln)
    assert (got == _oracle_md5(oracle, buf, off, ln)).all()
    assert (hc.crc32_messages(buf, off, ln) == oracle.crc32_messages(buf, off, ln)).all()


def test_md5_host_batch(cuda, oracle):
    """hc_md5_messages: host records through the pinned pipeline (several
    chunks: more records than one slot's 262144)."""
    rng = np.random.default_rng(4)
    n = 600_000
    lens = rng.integers(0, 200, n).astype(np.uint32)
    buf, off, ln = _packed(rng, lens, pad=1)
    got = M.md5_records(buf, off, ln)
    want = _oracle_md5(oracle, buf, off, ln)
    assert (got == want).all()


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 8, 1000, 65537, 1_000_001])
def test_merkle_levels_device(cuda, oracle, n):
    torch = cuda
    rng = np.random.default_rng(n)
    leaves = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    total = M.merkle_nodes(n)
    lv = torch.zeros(total * 16, dtype=torch.uint8, device="cuda")
    if n:
        lv[:n * 16] = torch.from_numpy(leaves.reshape(-1)).cuda()
    M.dev_merkle_levels(lv, n)
    torch.cuda.synchronize()
    levels = lv.cpu().numpy().reshape(-1, 16)
    tree = M.MerkleTree(levels, n)
    assert tree.root == oracle.merkle_root(leaves.tobytes())
    if n <= 65537:
        assert tree.Serialize() == oracle.merkle_serialize(leaves.tobytes())
    # the host entry (GPU from 65536 leaves) gives the same levels
    assert (M.NewMerkleTree(leaves, hashed_already=True).levels == levels).all()


def test_check_integrity_gpu(cuda, oracle):
    """CheckIntegrity's data half: 300k records -> GPU leaves -> tree -> Validate
    against the stored serialization; then one record corrupted: invalid, and
    DeepValidate's pair names that record (hashToOffset)."""
    rng = np.random.default_rng(5)
    n = 300_000
    lens = rng.integers(1, 600, n).astype(np.uint32)
    buf, off, ln = _packed(rng, lens, pad=0)
    leaves = _oracle_md5(oracle, buf, off, ln)
    stored = oracle.merkle_serialize(leaves.tobytes())
    ok, where = M.check_integrity(buf, off, ln, stored)
    assert ok and where == []
    for victim in (0, n - 1):
        bad = buf.copy()
        bad[int(off[victim]) + int(ln[victim]) // 2] ^= 0x40
        ok, where = M.check_integrity(bad, off, ln, stored)
        want = oracle.merkle_validate(_oracle_md5(oracle, bad, off, ln).tobytes(), stored)
        assert not ok and want[0] is False
        # Deserialize builds a left chain, so DeepValidate names a leaf only when
        # the chain's end meets the built tree's leftmost leaf; the oracle decides
        bad_leaves = _oracle_md5(oracle, bad, off, ln)
        named = {bad_leaves[i].tobytes(): i for i in range(n)}
        assert where == [named[h1] for h1, _h2 in want[1]], (victim, where)
