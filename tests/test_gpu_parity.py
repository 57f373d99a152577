"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, bit-exact.

Sizes: BASELINE.json configs 1-3 and the north-star 1M x 8 KiB at full size
(the oracle checks every CRC word, threaded), plus the edge cases the
reference path has: lengths 0..3 ("invalid block data"), unaligned blocks,
lengths that are not multiples of the 1 KiB row, whole-message CRCs, corrupt
blocks (verify bitmap / first bad index), in-place stamping and WAL-framed
blocks (lsm/wal/wal.go:177-271).
"""
import ctypes
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x48756E64


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def dev_uniform(torch, hc, seed, n, size):
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(buf, seed, stride=size, ulen=size, nblocks=n)
    return buf


def dev_crc(torch, hc, buf, n, **kw):
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, out, nblocks=n, **kw)
    torch.cuda.synchronize()
    return u32(out)


def test_zero_payload_known_answers(cuda, hc, golden):
    torch = cuda
    for B, want in golden["known"]["zero_payload"].items():
        B = int(B)
        buf = torch.zeros(1000 * B, dtype=torch.uint8, device="cuda")
        got = dev_crc(torch, hc, buf, 1000, stride=B, ulen=B)
        assert (got == want).all(), B
        assert hc.last_launch()["kernel"] == "k_crc_grp"


def test_config1_golden(cuda, hc, golden):
    torch = cuda
    c = golden["config1"]
    buf = dev_uniform(torch, hc, c["seed"], c["n"], c["block"])
    import hashlib
    assert hashlib.sha256(buf.cpu().numpy().tobytes()).hexdigest() == c["sha256_inputs"]
    got = dev_crc(torch, hc, buf, c["n"], stride=c["block"], ulen=c["block"])
    assert got.tolist() == c["crcs"]


@pytest.mark.parametrize("size", [4096, 8192, 16384])
def test_full_size_uniform(cuda, hc, oracle, size):
    """configs[1] (1M x 4 KiB) and the north star (1M x 8 KiB) at full size;
    16 KiB at 0.5M blocks.  Every word checked against the oracle."""
    torch = cuda
    n = 1_000_000 if size <= 8192 else 500_000
    buf = dev_uniform(torch, hc, SEED + size, n, size)
    got = dev_crc(torch, hc, buf, n, stride=size, ulen=size)
    host = buf.cpu().numpy()
    del buf
    want = oracle.crc32_blocks(host, stride=size, ulen=size, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}"


def test_config3_mixed_full(cuda, hc, oracle, golden):
    """configs[2]: 1M blocks, each 4/8/16 KiB (seeded), packed + off[]/len[]."""
    torch = cuda
    m = golden["mixed"]
    n = 1_000_000
    L = oracle.lib()
    sizes = np.array([L.oc_mixed_size(m["seed"], i) for i in range(n)], dtype=np.uint32)
    assert sizes[: m["n"]].tolist() == m["sizes"]
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    total = int(off[-1]) + int(sizes[-1])
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(sizes.view(np.int32)).cuda()
    hc.dev_fill_blocks(buf, m["seed"], off=doff, lens=dlen, nblocks=n)
    got = dev_crc(torch, hc, buf, n, off=doff, lens=dlen)
    assert got[: m["n"]].tolist() == m["crcs"]
    host = buf.cpu().numpy()
    del buf
    want = oracle.crc32_blocks(host, off=off, lens=sizes, threads=16)
    assert (got == want).all()


def test_general_lengths_and_alignment(cuda, hc, oracle):
    """Any length (0..70000, incl. <4) at any byte alignment; conforming blocks
    take the streaming kernel, the rest the general kernel, in one call."""
    torch = cuda
    rng = np.random.default_rng(21)
    n = 20000
    lens = rng.integers(0, 9000, n).astype(np.uint32)
    lens[:50] = np.arange(50)                     # tiny, incl. 0..3
    lens[50:2000] = 1024 * rng.integers(1, 17, 1950)  # conforming sizes ...
    lens[3000:3010] = 70000
    gaps = rng.integers(0, 64, n).astype(np.uint64)
    gaps[50:1000] = 0                              # ... some of them 16-B aligned
    off = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        if 50 <= i < 1000:
            pos = (pos + 15) & ~15
        off[i] = pos
        pos += int(lens[i])
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    got = dev_crc(torch, hc, buf, n, off=doff, lens=dlen)
    want = oracle.crc32_blocks(host, off=off, lens=lens, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], lens[bad[:10]], off[bad[:10]] % 16)


def test_small_messages_lane_parallel(cuda, hc, oracle):
    """Whole-message CRCs of records <= 1020 B are hashed one per lane (k_crc_any
    kVar bit 4): lengths 0..3, around the 1020/1021 threshold, any alignment,
    unsorted and overlapping offsets, records at offset 0 and empty records at
    the buffer's end, mixed with wave-path records -- vs the oracle."""
    torch = cuda
    rng = np.random.default_rng(1020)
    total = 8_000_000
    host = rng.integers(0, 256, total, dtype=np.uint8)
    n = 40_000
    kind = rng.integers(0, 10, n)
    lens = np.where(kind < 4, rng.integers(0, 64, n),
                    np.where(kind < 8, rng.integers(64, 1022, n), rng.integers(1021, 4000, n))).astype(np.uint32)
    lens[:40] = np.r_[np.arange(8), np.arange(1014, 1030), np.arange(16)]
    off = rng.integers(0, total - 4000, n).astype(np.uint64)  # unsorted, overlapping
    off[:5] = 0
    off[-5:] = total
    lens[-5:] = 0
    assert (off + lens <= total).all()  # every record inside the buffer before any launch
    buf = torch.from_numpy(host).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    got = dev_crc(torch, hc, buf, n, off=doff, lens=dlen, flags=hc.HC_F_MESSAGES)
    want = oracle.crc32_messages(host, off, lens, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], lens[bad[:10]], off[bad[:10]] % 16)
    # a batch of small records only, packed back to back at an odd address
    sl = rng.integers(0, 1021, 6_000).astype(np.uint32)
    so = np.zeros(sl.size, dtype=np.uint64)
    so[1:] = np.cumsum(sl[:-1], dtype=np.uint64)
    so += 1
    assert (so + sl <= total).all()
    dso = torch.from_numpy(so.view(np.int64)).cuda()
    dsl = torch.from_numpy(sl.view(np.int32)).cuda()
    got = dev_crc(torch, hc, buf, sl.size, off=dso, lens=dsl, flags=hc.HC_F_MESSAGES)
    assert (got == oracle.crc32_messages(host, so, sl, threads=16)).all()


@pytest.mark.parametrize("size,gap", [(1024, 0), (3072, 16), (5120, 0), (4096, 0), (4096, 16),
                                      (12288, 0), (20480, 48)])
def test_uniform_kernel_routes(cuda, hc, oracle, size, gap):
    """Uniform aligned batches: lengths that are multiples of 4 KiB take
    k_crc_grp (groups of 4 rows), other multiples of 1 KiB k_crc_fast; both
    bit-exact in block mode (CRC, stamp, verify with corruption) and in
    whole-message mode, including batches smaller than one block per wave."""
    torch = cuda
    stride = size + gap
    want_kernel = "k_crc_grp" if size % 4096 == 0 else "k_crc_fast"
    for n in (1, 7, 4095, 40_000):
        host = np.random.default_rng(size * 7 + n).integers(0, 256, n * stride, dtype=np.uint8)
        buf = torch.from_numpy(host).cuda()
        got = dev_crc(torch, hc, buf, n, stride=stride, ulen=size)
        assert hc.last_launch()["kernel"] == want_kernel
        want = oracle.crc32_blocks(host, stride=stride, ulen=size, nblocks=n, threads=16)
        assert (got == want).all(), (size, gap, n)
        off = np.arange(n, dtype=np.uint64) * stride
        lens = np.full(n, size, dtype=np.uint32)
        got = dev_crc(torch, hc, buf, n, stride=stride, ulen=size, flags=hc.HC_F_MESSAGES)
        assert hc.last_launch()["kernel"] == want_kernel
        assert (got == oracle.crc32_messages(host, off, lens, threads=16)).all(), (size, gap, n)
    # stamp in place, verify clean, corrupt, verify again (last n = 40000)
    hc.dev_crc32_blocks(buf, None, stride=stride, ulen=size, nblocks=n, flags=hc.HC_F_STAMP)
    stamped = buf.cpu().numpy()
    words = np.stack([stamped[i * stride:i * stride + 4] for i in range(n)]).copy().view("<u4").reshape(-1)
    assert (words == want).all()
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, stride=stride, ulen=size, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == 2**63 - 1 and int(bm.abs().sum().item()) == 0
    rng = np.random.default_rng(size + gap)
    victims = np.sort(rng.choice(n, 97, replace=False))
    pos = victims.astype(np.int64) * stride + rng.integers(0, size, victims.size)
    buf[torch.from_numpy(pos).cuda()] ^= 0x10
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, stride=stride, ulen=size, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == int(victims[0])
    bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(np.nonzero(bits)[0], victims)


def test_uniform_nonconforming_goes_general(cuda, hc, oracle):
    torch = cuda
    for size, stride in [(4100, 4100), (4096, 4100), (1000, 1000), (3, 8), (5000, 5008)]:
        n = 3000
        host = np.random.default_rng(size).integers(0, 256, n * stride + 16, dtype=np.uint8)
        buf = torch.from_numpy(host).cuda()
        got = dev_crc(torch, hc, buf, n, stride=stride, ulen=size)
        assert hc.last_launch()["kernel"] == "k_crc_any"
        want = oracle.crc32_blocks(host, stride=stride, ulen=size, nblocks=n)
        assert (got == want).all(), (size, stride)


def test_off_only_and_len_only(cuda, hc, oracle):
    """hundcrc.h lets a device batch pass only one of off[] / len[]: off[i]
    with the uniform length, or block i at i * stride with len[i].  Both go
    to k_crc_any (k_crc_grp takes both arrays or neither), in block mode,
    whole-message mode and verify mode."""
    torch = cuda
    rng = np.random.default_rng(29)
    n = 6000
    # off only: shuffled 4 KiB blocks (the shape k_crc_grp would take with len[])
    size = 4096
    host = rng.integers(0, 256, n * size + 64, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    off = (rng.permutation(n).astype(np.uint64) * size) + np.uint64(16)
    lens = np.full(n, size, dtype=np.uint32)
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    got = dev_crc(torch, hc, buf, n, off=doff, ulen=size)
    assert hc.last_launch()["kernel"] == "k_crc_any"
    assert (got == oracle.crc32_blocks(host, off=off, lens=lens, threads=16)).all()
    got = dev_crc(torch, hc, buf, n, off=doff, ulen=size, flags=hc.HC_F_MESSAGES)
    assert (got == oracle.crc32_messages(host, off, lens, threads=16)).all()
    # len only: block i at i * stride, any length up to the stride (0..3 incl.)
    stride = 9008
    lens = rng.integers(0, stride + 1, n).astype(np.uint32)
    lens[:8] = np.arange(8)
    lens[8:100] = 4096
    host = rng.integers(0, 256, n * stride, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    off = np.arange(n, dtype=np.uint64) * stride
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    got = dev_crc(torch, hc, buf, n, lens=dlen, stride=stride)
    assert hc.last_launch()["kernel"] == "k_crc_any"
    want = oracle.crc32_blocks(host, off=off, lens=lens, threads=16)
    assert (got == want).all()
    # verify with len only: every block clean except the ones under 4 bytes
    stamped = host.copy()
    for i in range(n):
        if lens[i] >= 4:
            stamped[i * stride:i * stride + 4] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    buf = torch.from_numpy(stamped).cuda()
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, lens=dlen, stride=stride, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(np.nonzero(bits)[0], np.nonzero(lens < 4)[0])
    assert int(fb.item()) == 0


def test_messages_mode(cuda, hc, oracle):
    """GetCRC over variable-length records (WAL records 64 B..64 KiB, config 5b)."""
    torch = cuda
    rng = np.random.default_rng(5)
    n = 30000
    lens = rng.integers(0, 66000, n).astype(np.uint32)
    lens[:40] = np.arange(40)
    lens[40:400] = 1024 * rng.integers(1, 40, 360)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 20, n - 1).astype(np.uint64))
    size = int(off[-1] + lens[-1]) + 32
    host = rng.integers(0, 256, size, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    got = dev_crc(torch, hc, buf, n, off=doff, lens=dlen, flags=hc.HC_F_MESSAGES)
    want = oracle.crc32_messages(host, off, lens, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], lens[bad[:10]])


def test_stamp_then_verify_and_corruption(cuda, hc, oracle):
    torch = cuda
    n, B = 200_000, 4096
    buf = dev_uniform(torch, hc, 99, n, B)
    hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, flags=hc.HC_F_STAMP)
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == 2**63 - 1 and int(bm.abs().sum().item()) == 0
    # stamped words equal the oracle's AddCRCToBlockData
    host = buf.cpu().numpy()
    want = oracle.crc32_blocks(host, stride=B, ulen=B, threads=16)
    assert (host.reshape(n, B)[:, :4].copy().view("<u4").reshape(-1) == want).all()
    # corrupt: one flipped bit in each chosen block (payload or stored word)
    rng = np.random.default_rng(8)
    victims = np.sort(rng.choice(n, 777, replace=False))
    pos = victims * B + rng.integers(0, B, victims.size)
    bits = rng.integers(0, 8, victims.size)
    idx = torch.from_numpy(pos.astype(np.int64)).cuda()
    flip = torch.from_numpy((1 << bits).astype(np.uint8)).cuda()
    buf[idx] ^= flip
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == int(victims[0])
    bits_set = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(np.nonzero(bits_set)[0], victims)


def test_wal_blocks_verify(cuda, hc, oracle):
    """Blocks framed exactly as lsm/wal/wal.go:177-271, verified as recoverMemtable does (:383)."""
    torch = cuda
    L = oracle.lib()
    sizes = np.array([L.oc_wal_record_size(3, i, 64, 65536) for i in range(4000)], dtype=np.uint32)
    blocks, st, _ = oracle.wal_frame(3, sizes)
    nb = st.blocks
    assert nb > 4000
    buf = torch.from_numpy(blocks).cuda()
    bm = torch.empty((nb + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, nb)
    hc.dev_crc32_blocks(buf, None, stride=4096, ulen=4096, nblocks=nb, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == 2**63 - 1
    buf[4096 * 17 + 4 + 17 + 10] ^= 1          # TestWAL_CorruptionDetection's byte (wal_test.go:884)
    hc.dev_verify_prepare(bm, fb, nb)
    hc.dev_crc32_blocks(buf, None, stride=4096, ulen=4096, nblocks=nb, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == 17


def test_host_entries(cuda, hc, oracle, golden):
    rng = np.random.default_rng(4)
    # uniform, packed
    host = rng.integers(0, 256, 5000 * 8192, dtype=np.uint8)
    assert (hc.crc32_blocks(host, stride=8192, ulen=8192) ==
            oracle.crc32_blocks(host, stride=8192, ulen=8192)).all()
    # mixed with arbitrary offsets and lengths
    lens = rng.integers(0, 20000, 3000).astype(np.uint32)
    off = rng.integers(0, host.size - 20000, 3000).astype(np.uint64)
    assert (hc.crc32_blocks(host, off=off, lens=lens) == oracle.crc32_blocks(host, off=off, lens=lens)).all()
    # messages
    assert (hc.crc32_messages(host, off, lens) == oracle.crc32_messages(host, off, lens)).all()
    # stamp + verify + corrupt
    blocks = rng.integers(0, 256, 3000 * 4096, dtype=np.uint8)
    hc.stamp_blocks(blocks)
    err, bm, fb = hc.verify_blocks(blocks)
    assert err is None and fb == -1 and bm.sum() == 0
    blocks[4096 * 1234 + 99] ^= 4
    blocks[4096 * 2000 + 7] ^= 1
    err, bm, fb = hc.verify_blocks(blocks)
    assert str(err) == "CRC mismatch in block" and fb == 1234
    assert np.nonzero(np.unpackbits(bm.view(np.uint8), bitorder="little"))[0].tolist() == [1234, 2000]
    # invalid (short) block in a batch
    err, bm, fb = hc.verify_blocks(blocks, off=np.array([0, 4096], np.uint64), lens=np.array([4096, 3], np.uint32))
    assert str(err) == "invalid block data" and fb == 1


def test_host_span_dma_pinned(cuda, hc, oracle):
    """off/len host batches in PINNED memory take the span-DMA path (one H2D
    copy of the byte span per chunk, no CPU gather): records back to back at an
    odd start, with small gaps, spanning several staging chunks; out-of-order
    and widely gapped offsets fall back to the gather path.  Every word vs the
    oracle; verify finds the corrupted block; md5 leaves vs the oracle."""
    torch = cuda
    from hunddb_amd import merkle as M
    rng = np.random.default_rng(41)
    n = 40_000
    lens = rng.integers(0, 9000, n).astype(np.uint32)
    gaps = np.where(rng.random(n) < 0.1, rng.integers(1, 40, n), 0).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    off += 3
    total = int(off[-1] + lens[-1]) + 64
    t = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    host = t.numpy()
    host[:] = rng.integers(0, 256, total, dtype=np.uint8)
    assert total > 2 * (64 << 20)  # several staging chunks
    want = oracle.crc32_messages(host, off, lens)
    assert (hc.crc32_messages(host, off, lens) == want).all()
    assert (hc.crc32_blocks(host, off=off, lens=lens) == oracle.crc32_blocks(host, off=off, lens=lens)).all()
    perm = rng.permutation(n)  # out of order: gather path
    assert (hc.crc32_messages(host, off[perm], lens[perm]) == want[perm]).all()
    wide = off * 3 // 2  # gaps of a third: gather path
    keep = wide + lens < total
    assert (hc.crc32_messages(host, wide[keep], lens[keep]) ==
            oracle.crc32_messages(host, wide[keep], lens[keep])).all()
    mw = np.empty((n, 16), np.uint8)
    oracle.lib().oc_md5_messages(host.ctypes.data, off.ctypes.data, lens.ctypes.data, mw.ctypes.data, n)
    assert (M.md5_records(host, off, lens) == mw).all()
    # 4 KiB blocks back to back in pinned memory, given as off/len: stamp, verify, corrupt
    nb = 20_000
    tb = torch.empty(nb * 4096, dtype=torch.uint8, pin_memory=True)
    blocks = tb.numpy()
    blocks[:] = rng.integers(0, 256, blocks.size, dtype=np.uint8)
    boff = np.arange(nb, dtype=np.uint64) * 4096
    blen = np.full(nb, 4096, np.uint32)
    hc.stamp_blocks(blocks, off=boff, lens=blen)
    err, bm, fb = hc.verify_blocks(blocks, off=boff, lens=blen)
    assert err is None and fb == -1
    blocks[4096 * 17_777 + 1000] ^= 0x80
    err, bm, fb = hc.verify_blocks(blocks, off=boff, lens=blen)
    assert str(err) == "CRC mismatch in block" and fb == 17_777


def test_add_crcs_to_data_gpu(cuda, hc, oracle):
    """AddCRCsToData (crc_util.go:41-64) over multi-hundred-block inputs runs on the GPU."""
    rng = np.random.default_rng(12)
    for n in [4092 * 256, 4092 * 1000 + 17, 3_000_001]:
        src = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out = hc.AddCRCsToData(src)
        want = np.zeros(hc.lib().hc_add_crcs_size(n), dtype=np.uint8)
        m = oracle.lib().oc_add_crcs_to_data(src, n, want.ctypes.data)
        assert m == len(out) and bytes(out) == want.tobytes()


@pytest.mark.default_thresholds
def test_default_thresholds_route(knobs, cuda, hc, oracle):
    """The production GPU/host crossovers (hc_util.hpp): an
    AddCRCsToData output, a ReadFromDisk and a WAL replay just below their
    threshold run on the host path, at it as one GPU batch (hc_stats), each
    byte-exact vs the oracle."""
    for k in ("HC_ADD_CRCS_GPU_MIN_BLOCKS", "HC_READ_GPU_MIN_BLOCKS", "HC_WAL_GPU_MIN_BLOCKS"):
        knobs.delenv(k, raising=False)
    rng = np.random.default_rng(31)
    for nb, gpu in ((2047, False), (2048, True)):
        n = nb * 4092 - 100  # nb output blocks, the last one ragged
        src = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        want = np.zeros(hc.lib().hc_add_crcs_size(n), dtype=np.uint8)
        assert oracle.lib().oc_add_crcs_to_data(src, n, want.ctypes.data) == len(want)
        hc.stats_reset()
        assert bytes(hc.AddCRCsToData(src)) == want.tobytes()
        st = hc.stats()
        assert (st["add_crcs_gpu"], st["add_crcs_host_small"]) == ((1, 0) if gpu else (0, 1)), nb
    B = 4096
    img = rng.integers(0, 256, 1100 * B, dtype=np.uint8)
    for i in range(1100):
        hc.AddCRCToBlockData(img[i * B:(i + 1) * B])
    for nb, gpu in ((1023, False), (1024, True)):
        size = nb * (B - 4)
        hc.stats_reset()
        got, fo, err = hc.ReadFromDisk(img.tobytes(), B, 4, size)
        want, wfo, wrc, _ = oracle.read_from_disk(img.tobytes(), B, 4, size)
        assert err is None and bytes(got) == bytes(want) and fo == wfo
        assert hc.stats()["read_gpu"] == (1 if gpu else 0), nb
    sizes = [oracle.lib().oc_wal_record_size(3, i, 64, 20000) for i in range(760)]
    wal, _, _ = oracle.wal_frame(3, sizes)
    wal = wal.tobytes()
    assert len(wal) // B >= 1024
    for nb, gpu in ((1023, False), (1024, True)):
        view = wal[:nb * B]
        hc.stats_reset()
        recs, err, bad, pos = hc.wal_replay(view, B)
        want, wrc, wbad, wpos = oracle.wal_replay(view, B, 0, 4, 0)
        assert recs == want and pos == wpos
        assert hc.stats()["wal_gpu"] == (1 if gpu else 0), nb


@pytest.mark.parametrize("inject", ["", "add_crcs", "add_crcs:nomem", "add_crcs:typo"])
def test_add_crcs_gpu_failure_finishes_on_host(knobs, cuda, hc, oracle, monkeypatch, inject):
    """VERDICT r3 weak 3 on the box: with a gfx950 present the multi-block
    AddCRCsToData is one GPU batch (hc_stats add_crcs_gpu); a failing batch
    (HC_INJECT_FAIL: HC_E_HIP / HC_E_NOMEM) is finished on the host path,
    byte-exact vs the oracle, counted as a fallback; HC_FORCE_GPU returns it.
    "<site>:<other suffix>" keeps the HC_E_HIP failure (it injected
    nothing in round 5)."""
    rng = np.random.default_rng(13)
    n = 4092 * 4000 + 333
    src = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    want = np.zeros(hc.lib().hc_add_crcs_size(n), dtype=np.uint8)
    assert oracle.lib().oc_add_crcs_to_data(src, n, want.ctypes.data) == len(want)
    if inject:
        knobs.setenv("HC_INJECT_FAIL", inject)
    hc.stats_reset()
    out = hc.AddCRCsToData(src)
    assert bytes(out) == want.tobytes()
    st = hc.stats()
    assert st["add_crcs_host_nodev"] == 0
    if inject:
        assert st["add_crcs_gpu_fallback"] == 1 and st["add_crcs_gpu"] == 0
        assert st["last_fallback_error"] == (hc.HC_E_NOMEM if "nomem" in inject else hc.HC_E_HIP)
        knobs.setenv("HC_FORCE_GPU", "1")
        with pytest.raises(hc.HundCRCError):
            hc.AddCRCsToData(src)
    else:
        assert st["add_crcs_gpu"] == 1 and st["add_crcs_gpu_fallback"] == 0


@pytest.mark.parametrize("mem", ["pageable", "pinned"])
def test_add_crcs_to_data_gpu_sources(cuda, hc, oracle, mem):
    """hc_add_crcs frames dst on host threads while the GPU hashes the SOURCE
    payload as 4092-byte messages (span DMA when src is pinned, CPU gather when
    pageable); the ragged last block is hashed on the host.  Byte-exact vs the
    oracle's crc_util.go:41-64 restatement: an exact multiple of 4092 (no ragged
    block), odd source addresses, and 70 MB spanning several staging chunks."""
    torch = cuda
    rng = np.random.default_rng(21)
    for n, shift in [(4092 * 300, 0), (4092 * 777, 3), (4092 * 300 + 4091, 1), (70_000_003, 5)]:
        if mem == "pinned":
            t = torch.empty(n + shift, dtype=torch.uint8, pin_memory=True)
            buf = t.numpy()
        else:
            buf = np.empty(n + shift, dtype=np.uint8)
        src = buf[shift:]
        src[:] = rng.integers(0, 256, n, dtype=np.uint8)
        out = hc.AddCRCsToData(src)
        want = np.zeros(hc.lib().hc_add_crcs_size(n), dtype=np.uint8)
        m = oracle.lib().oc_add_crcs_to_data(src.tobytes(), n, want.ctypes.data)
        assert m == len(out) and bytes(out) == want.tobytes(), (mem, n, shift)


@pytest.mark.parametrize("B", [4096, 8192, 5000])
def test_read_from_disk_gpu_copyout_shapes(knobs, cuda, hc, oracle, monkeypatch, B):
    """ReadFromDisk's payload copy-out runs on HC_COPY_THREADS threads while the
    GPU batch verifies; every block's output position comes from a closed form.
    Odd start offsets, sizes ending mid-block, images shorter than the touched
    range (zero-extended blocks), 1 and 3 copy threads, vs the oracle."""
    rng = np.random.default_rng(B)
    img = _stamped_blocks(oracle, rng, 1200, B)
    for threads in ["1", "3"]:
        knobs.setenv("HC_COPY_THREADS", threads)
        for start, size, cut in [(0, 1100 * (B - 4) + 333, 0), (7, 1000 * (B - 4), 0), (B + 123, 900 * (B - 4) + 1, 0),
                                 (4, 1150 * (B - 4), B * 60 + 77)]:
            view = img[(start // B) * B:].tobytes()
            if cut:
                view = view[:len(view) - cut]
            got, fo, err = hc.ReadFromDisk(view, B, start, size)
            want, wfo, wrc, wbad = oracle.read_from_disk(view, B, start, size)
            assert (0 if err is None else err.code) == wrc, (threads, start, size, cut)
            if wrc == 0:
                assert got == want and fo == wfo, (threads, start, size, cut)
            else:
                assert hc.last_bad_block() == wbad


def test_force_gpu_dropins(knobs, cuda, hc, golden, monkeypatch):
    knobs.setenv("HC_FORCE_GPU", "1")
    assert hc.GetCRC(b"123456789") == 0xCBF43926
    for v in golden["known"]["vectors"]:
        if v["hex"] is not None:
            assert hc.GetCRC(bytes.fromhex(v["hex"])) == v["crc"]
    for c in golden["functions"]["add_crc_to_block_data"]:
        b = bytearray.fromhex(c["in"])
        hc.AddCRCToBlockData(b)
        assert b.hex() == c["out"]
    for c in golden["functions"]["check_block_integrity"]:
        err = hc.CheckBlockIntegrity(bytes.fromhex(c["in"]))
        assert (None if err is None else str(err)) == c["err"]
    for c in golden["functions"]["fix_last_block_crc"]:
        b = bytearray.fromhex(c["in"])
        hc.FixLastBlockCRC(b)
        import hashlib
        assert hashlib.sha256(bytes(b)).hexdigest() == c["sha256"]


def test_concurrent_host_batches(cuda, hc, oracle):
    """Flush workers / compaction goroutines calling the batch entry at once."""
    rng = np.random.default_rng(6)
    datas = [rng.integers(0, 256, 2000 * 4096, dtype=np.uint8) for _ in range(6)]
    wants = [oracle.crc32_blocks(d) for d in datas]
    errors = []

    def work(i):
        for _ in range(3):
            if not (hc.crc32_blocks(datas[i]) == wants[i]).all():
                errors.append(i)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors


def test_concurrent_mixed_host_entries(cuda, hc, oracle):
    """Every host batch entry at once from 12 threads (3x the pipeline pool):
    CRC words, GPU-side verify (clean and corrupt), stamping as chunks retire,
    AddCRCsToData (framing overlapped with the source batch), ReadFromDisk
    (copy-out overlapped with the verify) and whole-message CRCs; every result
    against the oracle, the pool never above HC_MAX_PIPES."""
    rng = np.random.default_rng(61)
    B, nb = 4096, 3000
    data = rng.integers(0, 256, nb * B, dtype=np.uint8)
    words = oracle.crc32_blocks(data)
    stamped = _stamped_blocks(oracle, rng, nb, B)
    bad = stamped.copy()
    bad[1777 * B + 99] ^= 1
    payload = rng.integers(0, 256, 4092 * 600 + 123, dtype=np.uint8).tobytes()
    frame_want = np.zeros(hc.lib().hc_add_crcs_size(len(payload)), dtype=np.uint8)
    oracle.lib().oc_add_crcs_to_data(payload, len(payload), frame_want.ctypes.data)
    rd_want = oracle.read_from_disk(stamped.tobytes(), B, 7, 2900 * 4092)
    lens = rng.integers(0, 20000, 3000).astype(np.uint32)
    off = np.zeros(3000, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    msgs = rng.integers(0, 256, int(off[-1]) + int(lens[-1]) + 16, dtype=np.uint8)
    msg_want = oracle.crc32_messages(msgs, off, lens)
    errors = []

    def work(kind):
        try:
            for _ in range(3):
                if kind == 0:
                    assert (hc.crc32_blocks(data) == words).all()
                elif kind == 1:
                    err, _bm, fb = hc.verify_blocks(stamped)
                    assert err is None and fb == -1
                    err, bm, fb = hc.verify_blocks(bad)
                    assert str(err) == "CRC mismatch in block" and fb == 1777
                    assert np.nonzero(np.unpackbits(bm.view(np.uint8), bitorder="little"))[0].tolist() == [1777]
                elif kind == 2:
                    cp = stamped.copy()
                    cp.reshape(nb, B)[:, :4] = 0
                    hc.stamp_blocks(cp)
                    assert np.array_equal(cp, stamped)
                elif kind == 3:
                    assert bytes(hc.AddCRCsToData(payload)) == frame_want.tobytes()
                elif kind == 4:
                    got, fo, err = hc.ReadFromDisk(stamped.tobytes(), B, 7, 2900 * 4092)
                    assert err is None and got == rd_want[0] and fo == rd_want[1]
                else:
                    assert (hc.crc32_messages(msgs, off, lens) == msg_want).all()
        except AssertionError as e:  # noqa: PERF203
            errors.append((kind, repr(e)))

    ts = [threading.Thread(target=work, args=(i % 6,)) for i in range(12)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors, errors[:3]
    assert hc.host_pipelines() <= 4


def test_side_stream(cuda, hc, oracle):
    torch = cuda
    s = torch.cuda.Stream()
    n, B = 50_000, 8192
    with torch.cuda.stream(s):
        buf = torch.empty(n * B, dtype=torch.uint8, device="cuda")
        hc.dev_fill_blocks(buf, 77, stride=B, ulen=B, nblocks=n, stream=s)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        hc.dev_crc32_blocks(buf, out, stride=B, ulen=B, nblocks=n, stream=s)
    s.synchronize()
    host = buf.cpu().numpy()
    assert (u32(out) == oracle.crc32_blocks(host, stride=B, ulen=B, threads=16)).all()


@pytest.mark.parametrize("shift", [0, 1, 3, 4, 7, 13])
def test_dev_add_crcs_fused(cuda, hc, oracle, shift):
    """Fused framing + CRC (k_frame) vs the oracle's AddCRCsToData (crc_util.go:41-64),
    byte-exact, for ragged payload sizes around the 4092-byte boundary and
    unaligned payload starts."""
    torch = cuda
    rng = np.random.default_rng(100 + shift)
    for n in [1, 3, 4, 1019, 1020, 4091, 4092, 4093, 8184, 8185, 100_003, 4092 * 777 + 4090]:
        host = rng.integers(0, 256, n + shift, dtype=np.uint8)
        dsrc = torch.from_numpy(host).to("cuda")[shift:]
        assert dsrc.data_ptr() % 16 == shift % 16
        out_n = hc.lib().hc_add_crcs_size(n)
        dst = torch.full((out_n + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        crcs = torch.empty(out_n // 4096, dtype=torch.int32, device="cuda")
        hc.dev_add_crcs(dsrc, dst, crc_out=crcs, n=n)
        torch.cuda.synchronize()
        assert hc.last_launch()["kernel"] == "k_frame"
        got = dst.cpu().numpy()
        want = np.zeros(out_n, dtype=np.uint8)
        src = host[shift:].tobytes()
        assert oracle.lib().oc_add_crcs_to_data(src, n, want.ctypes.data) == out_n
        assert got[:out_n].tobytes() == want.tobytes(), n
        assert (got[out_n:] == 0xA5).all(), "wrote past the framed output"
        assert (u32(crcs) == want.view(np.uint32)[::1024]).all()


def test_dev_add_crcs_tiny_last_block(cuda, hc, oracle):
    """k_frame's interior blocks load aligned 16-B chunks, the last lane's second
    chunk through a buffer range that ends on the 16-B boundary after src's last
    byte: every source misalignment with a last block of 1-16 payload bytes, so
    the interior block before it reads right up to that boundary."""
    torch = cuda
    rng = np.random.default_rng(77)
    for shift in range(16):
        for tail in range(1, 17):
            n = 4092 * 3 + tail
            host = rng.integers(0, 256, n + shift, dtype=np.uint8)
            dsrc = torch.from_numpy(host).to("cuda")[shift:]
            out_n = hc.lib().hc_add_crcs_size(n)
            dst = torch.full((out_n,), 0xA5, dtype=torch.uint8, device="cuda")
            hc.dev_add_crcs(dsrc, dst, n=n)
            torch.cuda.synchronize()
            want = np.zeros(out_n, dtype=np.uint8)
            assert oracle.lib().oc_add_crcs_to_data(host[shift:].tobytes(), n, want.ctypes.data) == out_n
            assert dst.cpu().numpy().tobytes() == want.tobytes(), (shift, tail)


def test_dev_add_crcs_large_properties(cuda, hc, oracle):
    """256 MiB payload: the framed output's blocks verify clean, the payload
    round-trips (SizeWithoutCRCs direction), and the CRC words match the
    streaming kernel's CRCs of the same blocks."""
    torch = cuda
    n = 256 * 2**20 + 12345
    src = torch.empty(n + 3, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(src, 9, stride=n + 3, ulen=n + 3, nblocks=1)
    src = src[3:]
    dst = hc.dev_add_crcs(src)
    nb = dst.numel() // 4096
    crc_frame = torch.empty(nb, dtype=torch.int32, device="cuda")
    hc.dev_add_crcs(src, dst, crc_out=crc_frame)
    crc_stream = dev_crc(torch, hc, dst, nb, stride=4096, ulen=4096)
    assert (u32(crc_frame) == crc_stream).all()
    assert (dst.view(nb, 4096)[:, :4].contiguous().view(torch.int32).view(-1).cpu().numpy().view(np.uint32)
            == crc_stream).all()
    payload = dst.view(nb, 4096)[:, 4:].reshape(-1)
    assert torch.equal(payload[:n], src)
    assert int(payload[n:].count_nonzero()) == 0
    # spot-check a few blocks against the oracle's CRC
    idx = [0, 1, nb // 2, nb - 1]
    blocks = dst.view(nb, 4096)[idx].cpu().numpy()
    assert (oracle.crc32_blocks(blocks) == crc_stream[idx]).all()
    with pytest.raises(hc.HundCRCError):
        hc.dev_add_crcs(src[:5000], torch.empty(8192 + 16, dtype=torch.uint8, device="cuda")[1:])


def _stamped_blocks(oracle, rng, n, B):
    raw = rng.integers(0, 256, n * B, dtype=np.uint8)
    crcs = oracle.crc32_blocks(raw, stride=B, ulen=B)
    raw.view(np.uint32).reshape(n, B // 4)[:, 0] = crcs
    return raw


@pytest.mark.parametrize("B", [4096, 8192, 16384])
def test_dev_read_blocks_parity(cuda, hc, oracle, B):
    """k_unframe (batched ReadFromDisk, block_manager.go:203-235) vs the oracle:
    payloads byte-exact, CRC words, and the corrupt blocks found."""
    torch = cuda
    rng = np.random.default_rng(B)
    for n in [1, 2, 3, 17, 1000, 4099]:
        host = _stamped_blocks(oracle, rng, n, B)
        bad_idx = sorted(set(rng.integers(0, n, max(1, n // 300)).tolist())) if n > 2 else []
        for i in bad_idx:
            host[i * B + int(rng.integers(0, B))] ^= 1 << int(rng.integers(0, 8))
        want_crc = oracle.crc32_blocks(host, stride=B, ulen=B)
        stored = host.view(np.uint32).reshape(n, B // 4)[:, 0]
        want_bad = np.nonzero(stored != want_crc)[0]
        d = torch.from_numpy(host).to("cuda")
        bitmap = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
        fb = torch.empty(1, dtype=torch.int64, device="cuda")
        crcs = torch.empty(n, dtype=torch.int32, device="cuda")
        hc.dev_verify_prepare(bitmap, fb, n)
        out = torch.full((n * (B - 4) + 32,), 0x5A, dtype=torch.uint8, device="cuda")
        hc.dev_read_blocks(d, B, out=out, crc_out=crcs, bad_bitmap=bitmap, first_bad=fb)
        torch.cuda.synchronize()
        assert hc.last_launch()["kernel"] == "k_unframe"
        got = out.cpu().numpy()
        assert got[: n * (B - 4)].tobytes() == host.reshape(n, B)[:, 4:].tobytes(), (n, B)
        assert (got[n * (B - 4):] == 0x5A).all()
        assert (u32(crcs) == want_crc).all()
        bits = np.unpackbits(u32(bitmap).view(np.uint8), bitorder="little")[:n]
        assert np.nonzero(bits)[0].tolist() == want_bad.tolist()
        assert int(fb.item()) == (int(want_bad[0]) if len(want_bad) else 2**63 - 1)


@pytest.mark.parametrize("B", [4096, 8192, 16384])
@pytest.mark.parametrize("shift", [1, 2, 3, 4, 8, 12])
def test_dev_read_blocks_misaligned_out(cuda, hc, oracle, B, shift):
    """payload_out at any byte alignment (hundcrc.h: only `blocks` must be
    16-byte aligned): k_unframe's unaligned 16-B stores and, at 4 KiB, the
    12-B head store through a buffer range based at out + b (B-4) - 4.  The
    bytes on both sides of the payload stay untouched."""
    torch = cuda
    rng = np.random.default_rng(B + shift)
    n = 37
    host = _stamped_blocks(oracle, rng, n, B)
    want_crc = oracle.crc32_blocks(host, stride=B, ulen=B)
    d = torch.from_numpy(host).to("cuda")
    raw = torch.full((n * (B - 4) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    out = raw[shift:shift + n * (B - 4)]
    crcs = torch.empty(n, dtype=torch.int32, device="cuda")
    hc.dev_read_blocks(d, B, out=out, crc_out=crcs)
    torch.cuda.synchronize()
    got = raw.cpu().numpy()
    assert got[shift:shift + n * (B - 4)].tobytes() == host.reshape(n, B)[:, 4:].tobytes(), (B, shift)
    assert (got[:shift] == 0xA5).all() and (got[shift + n * (B - 4):] == 0xA5).all()
    assert (u32(crcs) == want_crc).all()


def test_frame_unframe_round_trip_full_size(cuda, hc):
    """1M blocks: AddCRCsToData (k_frame) then batched ReadFromDisk (k_unframe)
    gives back the payload, every block verifies, and the CRC words agree with
    the streaming kernel's."""
    torch = cuda
    n_blk = 1_000_000
    npay = n_blk * 4092 - 777
    raw = torch.empty(npay + 5, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(raw, 4242, stride=npay + 5, ulen=npay + 5, nblocks=1)
    src = raw[5:]
    framed = hc.dev_add_crcs(src)
    assert framed.numel() == n_blk * 4096
    bitmap = torch.empty((n_blk + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bitmap, fb, n_blk)
    pay = hc.dev_read_blocks(framed, 4096, bad_bitmap=bitmap, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == 2**63 - 1 and int(bitmap.count_nonzero()) == 0
    assert torch.equal(pay[:npay], src) and int(pay[npay:].count_nonzero()) == 0
    # corrupt three blocks of the framed image: exactly those are reported
    for i in (0, 123457, n_blk - 1):
        framed[i * 4096 + 4000] ^= 1
    hc.dev_verify_prepare(bitmap, fb, n_blk)
    hc.dev_read_blocks(framed, 4096, out=pay, bad_bitmap=bitmap, first_bad=fb)
    torch.cuda.synchronize()
    bits = np.unpackbits(u32(bitmap).view(np.uint8), bitorder="little")[:n_blk]
    assert np.nonzero(bits)[0].tolist() == [0, 123457, n_blk - 1] and int(fb.item()) == 0


def test_dev_read_blocks_16k_full_size(cuda, hc):
    torch = cuda
    n, B = 500_000, 16384
    buf = dev_uniform(torch, hc, 99, n, B)
    hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, flags=hc.HC_F_STAMP)
    bitmap = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bitmap, fb, n)
    pay = hc.dev_read_blocks(buf, B, bad_bitmap=bitmap, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == 2**63 - 1
    assert torch.equal(pay.view(n, B - 4), buf.view(n, B)[:, 4:])


def test_read_from_disk_gpu_batch(cuda, hc, oracle, monkeypatch):
    """hc_read_from_disk with >= 256 touched blocks verifies them in one GPU batch."""
    rng = np.random.default_rng(77)
    B = 4096
    img = _stamped_blocks(oracle, rng, 3000, B)
    for start, size, flip in [(5, 2000 * 4092, None), (4096 * 3 + 9, 2500 * 4092, 1700), (0, 3000 * 4092, 2999)]:
        view = bytearray(img[(start // B) * B:].tobytes())
        if flip is not None:
            view[flip * B + 77] ^= 0x10
        got, fo, err = hc.ReadFromDisk(bytes(view), B, start, size)
        want, wfo, wrc, wbad = oracle.read_from_disk(bytes(view), B, start, size)
        assert (0 if err is None else err.code) == wrc
        if wrc == 0:
            assert got == want and fo == wfo
        else:
            assert hc.last_bad_block() == wbad == flip


def test_wal_replay_gpu_batch(cuda, hc, oracle):
    """Row f3 at a size whose verify runs as one GPU batch: hc_wal_replay vs the
    oracle's sequential wal.go:362-455 restatement, clean, memtable-full and
    with a corrupt block in the middle."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import walgen
    plan = walgen.WalPlan(0x57414C, nrec=40_000)
    img = plan.render(0, plan.nblocks)
    nb = plan.nblocks
    assert nb > 10_000
    for start, mr, corrupt in [(0, 0, None), (3, 5000, None), (0, 0, nb // 2), (nb // 3, 0, nb - 1)]:
        view = img.copy()
        if corrupt is not None:
            view[corrupt * 4096 + 3000] ^= 0x40
        (buf, off, ln), err, bad, pos = hc.wal_replay(view, 4096, start, 4, mr, as_arrays=True)
        want, wrc, wbad, wpos = oracle.wal_replay(view.tobytes(), 4096, start, 4, mr)
        assert (0 if err is None else err.code) == wrc
        assert pos == wpos and bad == wbad and len(ln) == len(want)
        assert [int(x) for x in ln] == [len(w) for w in want]
        got = buf[: int(off[-1] + ln[-1])].tobytes() if len(ln) else b""
        assert got == b"".join(want)


@pytest.mark.parametrize("flags", [0, 2])
def test_offsets_beyond_2_and_4_GiB(cuda, hc, oracle, flags):
    """off/len batches whose offsets have bit 31 of the low word set, and exceed
    4 GiB: the per-entry metadata path of k_crc_grp / k_crc_any must widen
    offsets as unsigned 64-bit (blocks mode and whole-message mode)."""
    torch = cuda
    rng = np.random.default_rng(4242 + flags)
    total = 5 * 2**30 + 12345
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    n = 3000
    lens = rng.integers(64, 20000, n).astype(np.uint32)
    lens[: n // 3] = 8192                                   # conforming sizes for the streaming kernel
    bases = np.array([0, 2**31 - 70000, 2**31 + 16, 2**32 - 3_000_000, 2**32 + 48, total - 11_000_000],
                     dtype=np.uint64)
    offs = []
    for i in range(n):
        b = bases[i % len(bases)]
        offs.append(int(b) + (i // len(bases)) * 20480 + (0 if i < n // 3 else int(rng.integers(0, 7))))
    off = np.array(offs, dtype=np.uint64)
    assert (off + lens <= total).all() and ((off & 0xFFFFFFFF) >= 2**31).any() and (off >= 2**32).any()
    doff = torch.from_numpy(off.view(np.int64)).to("cuda")
    dlen = torch.from_numpy(lens.view(np.int32)).to("cuda")
    hc.dev_fill_blocks(buf, 77, off=doff, lens=dlen, nblocks=n)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n, flags=flags)
    torch.cuda.synchronize()
    got = u32(out)
    host = np.concatenate([buf[int(o):int(o) + int(l)].cpu().numpy() for o, l in zip(off, lens)])
    hoff = np.zeros(n, dtype=np.uint64)
    hoff[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    if flags:
        want = oracle.crc32_messages(host, hoff, lens)
    else:
        want = oracle.crc32_blocks(host, off=hoff, lens=lens)
    assert (got == want).all(), int((got != want).sum())


@pytest.mark.parametrize("path", ["fast", "general", "unframe"])
def test_verify_every_block_bad(cuda, hc, path):
    """A batch where EVERY block fails CheckBlockIntegrity (unstamped random
    blocks, e.g. a wiped or foreign file): every bitmap bit set, first_bad 0,
    and no serialisation of all waves on the first_bad word (each wave lowers
    it at most once) -- the all-bad launch stays within a small factor of a
    clean launch of the same batch timed in this process (no absolute bound:
    boxes differ by several percent)."""
    import time
    torch = cuda
    n, B = 1_000_000, 4096
    buf = dev_uniform(torch, hc, 4242, n, B)  # random stored words: all mismatch
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    out = torch.empty(n * (B - 4), dtype=torch.uint8, device="cuda") if path == "unframe" else None
    kw = dict(stride=B, ulen=B)
    if path == "general":  # off/len with every block 4 bytes short of a 1 KiB multiple -> k_crc_any
        kw = dict(off=torch.arange(n, dtype=torch.int64, device="cuda") * B,
                  lens=torch.full((n,), B - 4, dtype=torch.int32, device="cuda"))

    def run():
        hc.dev_verify_prepare(bm, fb, n)
        if path == "unframe":
            hc.dev_read_blocks(buf, B, out=out, bad_bitmap=bm, first_bad=fb)
        else:
            hc.dev_crc32_blocks(buf, None, nblocks=n, bad_bitmap=bm, first_bad=fb, **kw)

    def timed():
        run()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    dt_bad = timed()
    assert int(fb.item()) == 0
    bits = np.unpackbits(u32(bm).view(np.uint8), bitorder="little")[:n]
    assert int(bits.sum()) == n
    # the same batch stamped (every block verifies clean), timed the same way
    stamp_kw = kw if path != "unframe" else dict(stride=B, ulen=B)
    hc.dev_crc32_blocks(buf, None, nblocks=n, flags=hc.HC_F_STAMP, **stamp_kw)
    dt_clean = timed()
    assert int(fb.item()) == 2**63 - 1 and int(bm.count_nonzero()) == 0
    # before the once-per-wave rule the all-bad k_unframe pass took ~7x a clean one
    # (1M atomics on one word); allow 2x plus 0.5 ms of launch noise
    assert dt_bad < 2.0 * dt_clean + 5e-4, f"{path}: bad {dt_bad * 1e3:.2f} ms vs clean {dt_clean * 1e3:.2f} ms"


def test_config4_full_size_sampled_and_sharded(cuda, hc, oracle):
    """configs[3] at full size on one GPU: 16M x 8 KiB = 131 GB resident.
    The oracle re-generates ALL 16M blocks on the host by index (the fill is
    keyed by block index; 16 threads, 1 GiB slices) and checks every CRC word
    (crc_util.go:15-17,88-100); the index-sharded launches of 8
    ranks (hunddb_amd.shard.index_range, what bench.py --gpus 8 runs) give the
    same words as the whole batch; a stamp -> verify pass over all 131 GB finds
    exactly the blocks corrupted at far-apart indices (block offsets past 2^32
    and 2^36 bytes)."""
    import ctypes
    from hunddb_amd import shard
    torch = cuda
    n, B, seed = 16_000_000, 8192, 0x48756E64
    buf = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(buf, seed, stride=B, ulen=B, nblocks=n)
    whole = torch.empty(n, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, whole, stride=B, ulen=B, nblocks=n)
    assert hc.last_launch()["kernel"] == "k_crc_grp"
    parts = torch.empty(n, dtype=torch.int32, device="cuda")
    for r in range(8):
        lo, hi = shard.index_range(n, 8, r)
        hc.dev_crc32_blocks(buf[lo * B:hi * B], parts[lo:hi], stride=B, ulen=B, nblocks=hi - lo)
    torch.cuda.synchronize()
    assert torch.equal(whole, parts)
    got = u32(whole)
    per = (1 << 30) // B  # blocks per 1 GiB host slice
    host = np.empty(per * B, dtype=np.uint8)
    for lo in range(0, n, per):
        k = min(per, n - lo)
        oracle.fill_range(seed, lo, k, B, out=host, threads=16)
        want = oracle.crc32_blocks(host, stride=B, ulen=B, nblocks=k, threads=16)
        bad = np.flatnonzero(got[lo:lo + k] != want)
        assert bad.size == 0, (lo + bad[:8], got[lo + bad[:8]], want[bad[:8]])
    del host
    # stamp all, corrupt a few far-apart blocks, verify all
    hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, flags=hc.HC_F_STAMP)
    victims = [524_289, 8_388_609, n - 1]  # byte offsets > 2^32, > 2^36, the last block
    for v in victims:
        buf[v * B + 4000] ^= 1
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    assert int(fb.item()) == victims[0]
    bits = np.unpackbits(u32(bm).view(np.uint8), bitorder="little")[:n]
    assert np.nonzero(bits)[0].tolist() == victims
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("B", [1000, 5000])
def test_host_batches_length_not_16B_multiple(cuda, hc, oracle, B):
    """Uniform host batches whose block length is not a 16-B multiple, stride ==
    length, >= 256 blocks (the staging gather once copied such
    batches back to back while the kernel read them at 16-B aligned slots, so
    every block after the first got a wrong CRC).  HundDB accepts any
    BlockSize >= 1024 (utils/config/config.go:241).  hc_crc32_blocks,
    hc_stamp_blocks, hc_verify_blocks, hc_read_from_disk and hc_wal_replay at
    block size B, every word / byte vs the oracle."""
    rng = np.random.default_rng(B)
    n = 3000
    raw = rng.integers(0, 256, n * B, dtype=np.uint8)
    want = oracle.crc32_blocks(raw, stride=B, ulen=B)
    assert (hc.crc32_blocks(raw, stride=B, ulen=B) == want).all()
    blocks = raw.copy()
    hc.stamp_blocks(blocks, stride=B, ulen=B)
    assert (blocks.reshape(n, B)[:, :4].copy().view("<u4").reshape(-1) == want).all()
    err, bm, fb = hc.verify_blocks(blocks, stride=B, ulen=B)
    assert err is None and fb == -1
    bad = blocks.copy()
    bad[B * 1777 + 9] ^= 1
    err, bm, fb = hc.verify_blocks(bad, stride=B, ulen=B)
    assert str(err) == "CRC mismatch in block" and fb == 1777
    # ReadFromDisk over >= 256 blocks of block size B (block_manager.go:189-242)
    for start, size, img in [(7, 2000 * (B - 4), blocks), (B * 3 + 100, 2500 * (B - 4), blocks),
                             (0, 2999 * (B - 4), bad)]:
        view = img[(start // B) * B:].tobytes()
        got, fo, err = hc.ReadFromDisk(view, B, start, size)
        wpay, wfo, wrc, wbad = oracle.read_from_disk(view, B, start, size)
        assert (0 if err is None else err.code) == wrc
        if wrc == 0:
            assert got == wpay and fo == wfo
        else:
            assert hc.last_bad_block() == wbad
    # WAL recovery at block size B (wal.go:362-455), verify batch on the GPU
    L = oracle.lib()
    sizes = np.array([L.oc_wal_record_size(B, i, 64, 20000) for i in range(3000)], dtype=np.uint32)
    wal, st, _ = oracle.wal_frame(B, sizes, bs=B)
    assert st.blocks >= 256
    for corrupt in (None, st.blocks // 2):
        view = wal.copy()
        if corrupt is not None:
            view[corrupt * B + B // 2] ^= 0x40
        recs, err, badb, pos = hc.wal_replay(view, B, 0, 4, 0)
        wrecs, wrc, wbad, wpos = oracle.wal_replay(view.tobytes(), B, 0, 4, 0)
        assert (0 if err is None else err.code) == wrc and badb == wbad and pos == wpos
        assert recs == wrecs


def test_host_pipeline_pool_bounded(cuda, hc, oracle):
    """host batches lease a pipeline from a bounded pool
    (HC_MAX_PIPES, default 4) instead of one per OS thread: 16 threads calling
    the batch entries at once all get correct words and the number of live
    pipelines never exceeds the bound."""
    rng = np.random.default_rng(16)
    datas = [rng.integers(0, 256, 700 * 4096, dtype=np.uint8) for _ in range(16)]
    wants = [oracle.crc32_blocks(d) for d in datas]
    errors, peak = [], [0]

    def work(i):
        for _ in range(3):
            if not (hc.crc32_blocks(datas[i]) == wants[i]).all():
                errors.append(i)
            peak[0] = max(peak[0], hc.host_pipelines())

    ts = [threading.Thread(target=work, args=(i,)) for i in range(16)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors
    assert 1 <= hc.host_pipelines() <= 4 and peak[0] <= 4


def test_pinned_uniform_blocks_larger_than_staging(cuda, hc, oracle, tmp_path):
    """a pinned, densely packed uniform batch whose blocks are
    larger than one staging slot used to return HC_E_ARG from the direct-DMA
    path; such blocks are now hashed one at a time like gathered ones.  Run in a
    child process with HC_CHUNK_MB=1 (3 MiB blocks, pinned memory)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys; sys.path.insert(0, {root!r})
import numpy as np, torch
from hunddb_amd import crc as hc
from oracle import oracle as O
B, n = 3 << 20, 7
t = torch.empty(n * B, dtype=torch.uint8, pin_memory=True)
a = t.numpy(); a[:] = np.random.default_rng(3).integers(0, 256, a.size, dtype=np.uint8)
got = hc.crc32_blocks(a, stride=B, ulen=B)
assert (got == O.crc32_blocks(a, stride=B, ulen=B)).all()
hc.stamp_blocks(a, stride=B, ulen=B)
err, bm, fb = hc.verify_blocks(a, stride=B, ulen=B)
assert err is None and fb == -1
print("ok")
"""
    env = dict(os.environ, HC_CHUNK_MB="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_read_from_disk_verified_mask_gpu_batch(cuda, hc, oracle):
    """Row f1 with the cache's verified bits at GPU-batch size: the unmasked
    blocks go to the GPU as one off/len batch, masked ones are not hashed."""
    import importlib
    sys_path_tests = os.path.dirname(os.path.abspath(__file__))
    import sys
    sys.path.insert(0, sys_path_tests)
    ta = importlib.import_module("test_abi")
    for B in (4096, 8192, 5000):
        ta._read_mask_case(hc, oracle, 3000, B, B + 1)


def test_offlen_sweep_skip_flag(cuda, hc, oracle):
    """The k_crc_any sweep after an off/len k_crc_grp exits at once when
    k_crc_grp left it no block (Batch::skip_slot).  Calls that alternate
    between fully conforming batches and batches with one non-conforming block
    (first, middle, last, the only block; misaligned or a length that is not a
    4 KiB multiple) must all be exact; `out` is poisoned before each call, so a
    sweep that wrongly exits leaves the poison.  Then the same on two streams at
    once, and a captured graph replayed after its off[] changed under it."""
    torch = cuda
    rng = np.random.default_rng(77)
    n = 3000
    host = rng.integers(0, 256, n * 16384 + 4096, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    base_off = np.arange(n, dtype=np.uint64) * 16384
    base_len = (4096 * rng.integers(1, 5, n)).astype(np.uint32)

    def run(off, lens, stream=None, m=n):
        doff = torch.from_numpy(off[:m].view(np.int64)).cuda()
        dlen = torch.from_numpy(lens[:m].view(np.int32)).cuda()
        out = torch.full((m,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=m, stream=stream)
        return out, (doff, dlen)

    cases = []
    for pos in (0, n // 2, n - 1):
        for kind in ("misaligned", "short"):
            off, lens = base_off.copy(), base_len.copy()
            if kind == "misaligned":
                off[pos] += 3
            else:
                lens[pos] -= 100
            cases.append((off, lens, n))
    single_off, single_len = base_off.copy(), base_len.copy()
    single_off[0] += 5
    seq = [(base_off, base_len, n)]
    for c in cases:
        seq += [c, (base_off, base_len, n)]
    seq += [(single_off, single_len, 1), (base_off, base_len, 1)]
    for off, lens, m in seq:
        out, _ = run(off, lens, m=m)
        torch.cuda.synchronize()
        want = oracle.crc32_blocks(host, off=off[:m], lens=lens[:m], threads=16)
        assert (u32(out) == want).all(), (m, np.nonzero(u32(out) != want)[0][:5])

    # two streams: one conforming, one with a misaligned block, many rounds
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    off_b, len_b = cases[1][0], cases[1][1]
    want_a = oracle.crc32_blocks(host, off=base_off, lens=base_len, threads=16)
    want_b = oracle.crc32_blocks(host, off=off_b, lens=len_b, threads=16)
    keep = []
    for _ in range(8):
        keep.append((run(base_off, base_len, stream=s1), run(off_b, len_b, stream=s2)))
    torch.cuda.synchronize()
    for (oa, _), (ob, _) in keep:
        assert (u32(oa) == want_a).all() and (u32(ob) == want_b).all()

    # a graph captured on a conforming batch, replayed after one offset moved
    doff = torch.from_numpy(base_off.view(np.int64)).cuda()
    dlen = torch.from_numpy(base_len.view(np.int32)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n, stream=s)  # warm (tables, init)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n, stream=s)
    torch.cuda.synchronize()
    for off in (base_off, off_b, base_off, off_b):
        doff.copy_(torch.from_numpy(off.view(np.int64)))
        out.fill_(0x5A5A5A5A)
        g.replay()
        torch.cuda.synchronize()
        want = oracle.crc32_blocks(host, off=off, lens=base_len, threads=16)
        assert (u32(out) == want).all()
