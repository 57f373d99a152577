"""Seeded random layouts through the batch entries, against the oracle.

Each case draws a layout the reference's callers can produce or the C ABI
accepts: uniform blocks (4/8/16 KiB and any other length, any stride, any
start alignment), off/len blocks (4 KiB multiples mixed with arbitrary
lengths, gaps, unaligned starts, lengths 0-3, shuffled and overlapping
entries) and whole messages (packed back to back, or scattered).  Every case
runs the device entry (hc_dev_crc32_blocks, so k_crc_grp / k_crc_fast /
k_crc_any routing; the k_seg_* stream for message batches and, with
HC_SEG_MIN_BLOCKS=1 on half the uniform cases, for the uniform blocks
k_crc_grp refuses) and the host entry (the pipelined staging path), and compares
the words with the oracle.  Non-overlapping block cases are then stamped on
the device, compared byte for byte, corrupted at random blocks and verified:
bitmap and first_bad must name exactly the corrupted blocks plus every block
shorter than 4 bytes (crc_util.go:89-91)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# HC_FUZZ_SCALE=k runs k times as many seeds of every case family (the default
# seeds are the first ones of the larger set): a longer sweep on the box
SCALE = max(1, int(os.environ.get("HC_FUZZ_SCALE", "1")))
N_CASES = 192 * SCALE
MAX_BYTES = 24 << 20


def _len(rng):
    r = rng.random()
    if r < 0.45:
        return int(rng.choice([4096, 8192, 16384]))
    if r < 0.55:
        return int(rng.integers(0, 4))
    if r < 0.7:
        return 1024 * int(rng.integers(1, 20))
    return int(rng.integers(4, 20000))


def gen_case(seed):
    rng = np.random.default_rng(seed)
    kind = ["uniform", "offlen", "messages"][seed % 3]
    lead = int(rng.choice([0, 0, 0, int(rng.integers(1, 16))]))  # start alignment of the data
    if kind == "uniform":
        ulen = _len(rng)
        stride = ulen + int(rng.choice([0, 0, 16 * int(rng.integers(1, 8)), int(rng.integers(1, 64))]))
        stride = max(stride, 1)
        n = int(rng.integers(1, max(2, min(3000, MAX_BYTES // stride))))
        size = lead + stride * (n - 1) + ulen + 64
        off, lens = None, None  # blocks start at byte `lead` of the buffer
    else:
        n = int(rng.integers(1, 3000))
        lens = np.array([_len(rng) for _ in range(n)], dtype=np.uint32)
        while lens.sum() > MAX_BYTES:
            lens = lens[: len(lens) // 2]
        n = len(lens)
        packed = kind == "messages" and rng.random() < 0.5
        gaps = np.zeros(n, dtype=np.uint64) if packed else rng.integers(0, 40, n).astype(np.uint64)
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
        off += np.uint64(lead)
        size = int(off[-1]) + int(lens[-1]) + 64
        if kind == "offlen" and rng.random() < 0.3:  # shuffled order, some entries repeated
            perm = rng.permutation(n)
            off, lens = off[perm], lens[perm]
            k = max(1, n // 10)
            off[:k], lens[:k] = off[-k:], lens[-k:]
        stride = ulen = 0
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    return kind, buf, off, lens, stride, ulen, n, (lead if off is None else 0)


def _words(oracle, kind, buf, off, lens, stride, ulen, n):
    if kind == "messages":
        return oracle.crc32_messages(buf, off, lens)
    return oracle.crc32_blocks(buf, off=off, lens=lens, stride=stride or 1, ulen=ulen, nblocks=n)


def _dev(torch, a):
    return None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(
        np.int64 if a.dtype == np.uint64 else np.int32)).cuda()


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_layout(knobs, cuda, hc, oracle, seed, monkeypatch):
    torch = cuda
    kind, buf, off, lens, stride, ulen, n, lead = gen_case(1000 + seed)
    packed = kind == "messages" and n > 1 and bool(
        np.all(off[1:] == off[:-1] + lens[:-1].astype(np.uint64)))
    if packed and seed % 2:
        knobs.setenv("HC_SEG_MIN_MSGS", "1")  # the packed-record stream on a small batch
    if kind == "uniform" and seed % 2:
        knobs.setenv("HC_SEG_MIN_BLOCKS", "1")  # blocks k_crc_grp refuses: the message stream (round 5)
    want = _words(oracle, kind, buf[lead:], off, lens, stride, ulen, n)
    flags = hc.HC_F_MESSAGES if kind == "messages" else 0
    # device entry
    dall = torch.from_numpy(buf).cuda()
    dbuf = dall[lead:]
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(dbuf, out, off=_dev(torch, off), lens=_dev(torch, lens), stride=stride, ulen=ulen,
                        nblocks=n, flags=flags)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want), (kind, int(np.flatnonzero(got != want)[0]), hc.last_launch())
    # host entry
    if kind == "messages":
        got_h = hc.crc32_messages(buf, off, lens)
    else:
        got_h = hc.crc32_blocks(buf[lead:], off=off, lens=lens, stride=stride, ulen=ulen, nblocks=n)
    assert np.array_equal(got_h, want), kind
    if kind == "messages":
        return
    # stamp + verify on the device (blocks must not overlap for a stamp)
    if off is not None:
        o = off.astype(np.int64)
        order = np.argsort(o, kind="stable")
        ends = o[order] + lens[order].astype(np.int64)
        if np.any(o[order][1:] < ends[:-1]) or len(np.unique(o)) != len(o):
            return
    rng = np.random.default_rng(seed)
    hc.dev_crc32_blocks(dbuf, None, off=_dev(torch, off), lens=_dev(torch, lens), stride=stride, ulen=ulen,
                        nblocks=n, flags=hc.HC_F_STAMP)
    torch.cuda.synchronize()
    ref = buf.copy()
    offs = off.astype(np.int64) if off is not None else lead + np.arange(n, dtype=np.int64) * stride
    L = lens if lens is not None else np.full(n, ulen, dtype=np.uint32)
    for i in range(n):
        if L[i] >= 4:
            ref[offs[i]:offs[i] + 4] = np.array([want[i]], dtype=np.uint32).view(np.uint8)
    assert np.array_equal(dall.cpu().numpy(), ref), kind
    bad = set(int(i) for i in np.flatnonzero(L < 4))
    cand = np.flatnonzero(L >= 5)
    for i in rng.choice(cand, size=min(len(cand), int(rng.integers(0, 4))), replace=False) if len(cand) else []:
        pos = int(offs[i]) + int(rng.integers(4, int(L[i])))
        dall[pos] ^= 0x40
        bad.add(int(i))
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(dbuf, None, off=_dev(torch, off), lens=_dev(torch, lens), stride=stride, ulen=ulen,
                        nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    bits = np.flatnonzero(np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little"))
    assert sorted(bits.tolist()) == sorted(bad), kind
    assert int(fb.item()) == (min(bad) if bad else 2**63 - 1)


N_FRAMING = 48 * SCALE


@pytest.mark.parametrize("seed", range(N_FRAMING))
def test_random_framing_round_trip(cuda, hc, oracle, seed):
    """AddCRCsToData (host entry: a GPU batch at or above the GPU tests' 256-block
    threshold -- conftest.py; production's is 2048 --, the host below it; device
    entry k_frame) on random payload sizes at random alignments, byte-exact vs
    the oracle; then ReadFromDisk over the framed image (host entry and the
    device k_unframe) at random start offsets and sizes, vs the oracle's
    block_manager.go:189-242 restatement, with one corrupted block in half the
    cases."""
    torch = cuda
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.choice([0, 1, 4091, 4092, 4093, int(rng.integers(1, 200 * 4092)),
                        int(rng.integers(256 * 4092, 1200 * 4092))]))
    lead = int(rng.integers(0, 16))
    raw = rng.integers(0, 256, n + lead + 16, dtype=np.uint8)
    pay = raw[lead:lead + n]
    want = np.zeros(hc.hc_add_crcs_size_py(n), dtype=np.uint8)
    if n:
        oracle.lib().oc_add_crcs_to_data(pay.ctypes.data, n, want.ctypes.data)
    got = np.frombuffer(bytes(hc.AddCRCsToData(pay)), dtype=np.uint8)
    assert np.array_equal(got, want)
    if n:
        dsrc = torch.from_numpy(raw).cuda()[lead:lead + n]
        framed = hc.dev_add_crcs(dsrc)
        torch.cuda.synchronize()
        assert np.array_equal(framed.cpu().numpy(), want)
    if len(want) == 0:
        return
    nb = len(want) // 4096
    img = want.copy()
    bad_blk = None
    if seed % 2 and nb > 1:
        bad_blk = int(rng.integers(0, nb))
        img[bad_blk * 4096 + int(rng.integers(4, 4096))] ^= 0x08
    # device k_unframe over the whole image
    dimg = torch.from_numpy(img).cuda()
    bm = torch.empty((nb + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, nb)
    payload = hc.dev_read_blocks(dimg, 4096, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == (bad_blk if bad_blk is not None else 2**63 - 1)
    if bad_blk is None:
        assert np.array_equal(payload.cpu().numpy()[:n], pay)
    # host ReadFromDisk at random offsets and sizes
    for _ in range(3):
        start = int(rng.integers(0, len(img)))
        size = int(rng.integers(0, max(1, len(img) - start)))
        b0 = start // 4096
        blocks = img[b0 * 4096:].tobytes()
        w_pay, w_fo, w_rc, w_bad = oracle.read_from_disk(blocks, 4096, start, size)
        g_pay, g_fo, g_err = hc.ReadFromDisk(blocks, 4096, start, size)
        if w_rc == 0:
            assert g_err is None and g_pay == w_pay and g_fo == w_fo
        else:
            assert g_err is not None and int(g_err.code) == w_rc and hc.last_bad_block() == w_bad


N_WAL = 24 * SCALE


@pytest.mark.parametrize("seed", range(N_WAL))
def test_random_wal_replay(cuda, hc, oracle, seed):
    """Row f3 with the GPU verify (>= 256 blocks): random record-size laws,
    block sizes 4096/8192/5000 (any BlockSize >= 1024 is valid, config.go:241),
    start blocks, memtable-full stops and corrupted blocks, against the
    oracle's sequential wal.go:362-455 restatement."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import walgen
    rng = np.random.default_rng(7000 + seed)
    bs = int(rng.choice([4096, 4096, 8192, 5000]))
    hi = int(rng.choice([2000, 20000, 65536]))
    plan = walgen.WalPlan(9000 + seed, nrec=int(rng.integers(1500, 6000)), lo=int(rng.choice([17, 64])), hi=hi, bs=bs)
    img = plan.render(0, plan.nblocks)
    nb = plan.nblocks
    for _ in range(3):
        view = img.copy()
        for k in range(int(rng.integers(0, 3))):
            blk = int(rng.integers(0, nb))
            view[blk * bs + int(rng.integers(4, bs))] ^= 1 << int(rng.integers(0, 8))
        start = int(rng.choice([0, 0, int(rng.integers(0, nb))]))
        mr = int(rng.choice([0, 0, int(rng.integers(1, 4000))]))
        (buf, off, ln), err, bad, pos = hc.wal_replay(view, bs, start, 4, mr, as_arrays=True)
        want, wrc, wbad, wpos = oracle.wal_replay(view.tobytes(), bs, start, 4, mr)
        assert (0 if err is None else err.code) == wrc, (bs, start, mr)
        assert pos == wpos and bad == wbad and len(ln) == len(want)
        got = buf[: int(off[-1] + ln[-1])].tobytes() if len(ln) else b""
        assert [int(x) for x in ln] == [len(w) for w in want]
        assert got == b"".join(want)


N_READ = 16 * SCALE


@pytest.mark.parametrize("seed", range(N_READ))
def test_random_read_from_disk_verified_mask(cuda, hc, oracle, seed):
    """Row f1 with the block cache's verified bits, random block sizes, start
    offsets, sizes, mask densities and corruptions (in masked and unmasked
    blocks), at GPU-batch sizes: the first unmasked corrupt block stops the read,
    masked blocks are trusted and never hashed, and a clean read returns what the
    oracle returns for the same bytes with the trusted blocks re-stamped."""
    rng = np.random.default_rng(8000 + seed)
    B = int(rng.choice([4096, 8192, 5000, 1024, 16384]))
    n = int(rng.integers(256, 4000 if B <= 8192 else 1500))
    raw = rng.integers(0, 256, n * B, dtype=np.uint8)
    raw.view(np.uint8).reshape(n, B)[:, :4] = oracle.crc32_blocks(raw, stride=B, ulen=B).view(
        np.uint8).reshape(n, 4)
    start = int(rng.integers(0, 3 * B))
    b0 = start // B
    size = int(rng.integers(1, (n - b0 - 1) * (B - 4)))
    k = hc.read_blocks_touched(B, start, size)
    blocks = raw[b0 * B:].copy()
    masked = rng.random(k) < float(rng.choice([0.0, 0.3, 0.9]))
    corrupt = sorted(set(int(x) for x in rng.integers(0, k, int(rng.integers(0, 4)))))
    for c in corrupt:
        blocks[c * B + int(rng.integers(4, B))] ^= 0x10
    v = np.zeros((k + 31) // 32, np.uint32)
    for i in np.flatnonzero(masked):
        v[i >> 5] |= np.uint32(1 << (int(i) & 31))
    got, fo, err = hc.ReadFromDisk(blocks.tobytes(), B, start, size, verified=v)
    live_bad = [c for c in corrupt if not masked[c]]
    assert hc.last_hashed() == int((~masked).sum())
    if live_bad:
        assert str(err) == "CRC mismatch in block" and hc.last_bad_block() == live_bad[0]
        return
    assert err is None
    fixed = blocks.copy()  # the trusted (masked) corrupt blocks re-stamped: the oracle accepts them
    fixed.reshape(-1, B)[:, :4] = oracle.crc32_blocks(fixed, stride=B, ulen=B).view(np.uint8).reshape(-1, 4)
    want, wfo, wrc, _ = oracle.read_from_disk(fixed.tobytes(), B, start, size)
    assert wrc == 0 and got == want and fo == wfo
    assert np.unpackbits(v.view(np.uint8), bitorder="little")[:k].sum() == k


N_MULTI = 16 * SCALE


@pytest.mark.parametrize("seed", range(N_MULTI))
def test_random_multi_gpu_plans(cuda, hc, oracle, seed):
    """The single-process multi-GPU entries on random block layouts and random
    plans (every range on device 0 of the one-GPU box, each on its own thread
    and pipeline): CRC words, and verify merged over the ranges, vs the oracle."""
    kind, buf, off, lens, stride, ulen, n, lead = gen_case(3000 + 3 * seed + (seed % 2))  # uniform / off-len
    if kind == "messages":
        kind, buf, off, lens, stride, ulen, n, lead = gen_case(3000 + 3 * seed + 1)
    rng = np.random.default_rng(seed)
    ndev = int(rng.integers(1, 9))
    if rng.random() < 0.5:
        cuts = np.sort(rng.integers(0, n + 1, ndev - 1))
        bounds = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    else:
        bounds = None  # hc_shard_plan
    base = buf[lead:]
    want = oracle.crc32_blocks(base, off=off, lens=lens, stride=stride or 1, ulen=ulen, nblocks=n)
    got = hc.multi_crc32_blocks(base, [0] * ndev, off=off, lens=lens, stride=stride, ulen=ulen, nblocks=n,
                                bounds=bounds)
    assert np.array_equal(got, want), (kind, ndev)
    err1, bm1, fb1 = hc.verify_blocks(base, off=off, lens=lens, stride=stride, ulen=ulen, nblocks=n)
    err, bm, fb = hc.multi_verify_blocks(base, [0] * ndev, off=off, lens=lens, stride=stride, ulen=ulen, nblocks=n,
                                         bounds=bounds)
    assert np.array_equal(bm, bm1) and fb == fb1 and str(err) == str(err1)


N_UNFRAME = 24 * SCALE


@pytest.mark.parametrize("seed", range(N_UNFRAME))
def test_random_dev_read_blocks(cuda, hc, oracle, seed):
    """Row f1 on the device at every block size (k_unframe: one wave per 4 KiB
    block; one wave per 4 KiB group of an 8/16 KiB block, the groups combined
    through LDS): random block counts (odd ones leave part of the last
    workgroup idle), random corruption (none, one, several, the first, the
    last, every block), against the oracle's CRCs: payload bytes, CRC words,
    the verify bitmap and first_bad."""
    torch = cuda
    rng = np.random.default_rng(9000 + seed)
    B = [4096, 8192, 16384][seed % 3]
    n = int(rng.choice([1, 2, 3, 5, int(rng.integers(1, 64)), int(rng.integers(64, 3000))]))
    raw = rng.integers(0, 256, n * B, dtype=np.uint8)
    raw.view(np.uint32).reshape(n, B // 4)[:, 0] = oracle.crc32_blocks(raw, stride=B, ulen=B)
    mode = seed % 6
    if mode == 1:
        bad = [int(rng.integers(0, n))]
    elif mode == 2:
        bad = sorted(set(rng.integers(0, n, 1 + n // 50).tolist()))
    elif mode == 3:
        bad = [0]
    elif mode == 4:
        bad = [n - 1]
    elif mode == 5:
        bad = list(range(n))
    else:
        bad = []
    for i in bad:  # a flipped bit anywhere in the block: payload or the stored word
        raw[i * B + int(rng.integers(0, B))] ^= 1 << int(rng.integers(0, 8))
    want = oracle.crc32_blocks(raw, stride=B, ulen=B)
    stored = raw.view(np.uint32).reshape(n, B // 4)[:, 0]
    want_bad = np.nonzero(stored != want)[0]
    d = torch.from_numpy(raw).cuda()
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    crcs = torch.empty(n, dtype=torch.int32, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    out = torch.full((n * (B - 4) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    hc.dev_read_blocks(d, B, out=out, crc_out=crcs, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert got[: n * (B - 4)].tobytes() == raw.reshape(n, B)[:, 4:].tobytes()
    assert (got[n * (B - 4):] == 0xA5).all()
    assert (crcs.cpu().numpy().view(np.uint32) == want).all()
    bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    assert np.nonzero(bits)[0].tolist() == want_bad.tolist()
    assert int(fb.item()) == (int(want_bad[0]) if len(want_bad) else 2**63 - 1)
