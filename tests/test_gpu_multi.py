"""GPU parity of the single-process multi-GPU entries (hc_multi_*,
hc_dev_multi_crc32_blocks) against the oracle and the one-GPU entries.  The box
has one GPU, so the shards of a plan all name device 0: every shard still runs
on its own thread through its own host pipeline, and the results are merged
exactly as with distinct devices."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def blocks(oracle, n, size, seed=0x77):
    buf, off, lens = oracle.fill_blocks(seed, n, size)
    return buf


@pytest.mark.parametrize("ndev", [1, 3, 4])
def test_multi_crc_uniform_vs_oracle(cuda, hc, oracle, ndev):
    n, B = 20_001, 4096
    buf = blocks(oracle, n, B)
    want = oracle.crc32_blocks(buf, stride=B, ulen=B)
    got = hc.multi_crc32_blocks(buf, [0] * ndev, stride=B, ulen=B)
    assert np.array_equal(got, want)
    # an explicit plan whose bounds are not multiples of 32 (nor of anything)
    b = np.array([0] + [1, 33, 4099, 12345][: ndev - 1] + [n], dtype=np.uint64)
    got = hc.multi_crc32_blocks(buf, [0] * ndev, stride=B, ulen=B, bounds=b)
    assert np.array_equal(got, want)


def test_multi_crc_offlen_mixed_vs_oracle(cuda, hc, oracle):
    rng = np.random.default_rng(5)
    lens = rng.choice([4096, 8192, 16384, 1000, 3], 6000).astype(np.uint32)
    buf, off, lens = oracle.fill_blocks(0x99, len(lens), sizes=lens)
    want = oracle.crc32_blocks(buf, off=off, lens=lens)
    got = hc.multi_crc32_blocks(buf, [0, 0, 0], off=off, lens=lens)  # plan balanced by bytes
    assert np.array_equal(got, want)
    assert np.array_equal(got, hc.crc32_blocks(buf, off=off, lens=lens))


def test_multi_verify_merges_shards(cuda, hc, oracle):
    n, B = 9_000, 8192
    buf = blocks(oracle, n, B)
    hc.stamp_blocks(buf, stride=B, ulen=B)
    err, bm, fb = hc.multi_verify_blocks(buf, [0, 0, 0, 0], stride=B, ulen=B)
    assert err is None and fb == -1 and not bm.any()
    bad = [8999, 6000, 2251, 4500, 2250]  # shards 3, 2, 1, 2, 0 of the 4-way plan
    for k in bad:
        buf[k * B + 100] ^= 0x01
    err, bm, fb = hc.multi_verify_blocks(buf, [0, 0, 0, 0], stride=B, ulen=B)
    assert fb == min(bad) and err is not None and str(err) == "CRC mismatch in block"
    err1, bm1, fb1 = hc.verify_blocks(buf, stride=B, ulen=B)
    assert np.array_equal(bm, bm1) and fb1 == fb
    bits = np.flatnonzero(np.unpackbits(bm.view(np.uint8), bitorder="little"))
    assert sorted(bits.tolist()) == sorted(bad)


def test_multi_verify_short_block_reason(cuda, hc, oracle):
    lens = np.full(3000, 4096, dtype=np.uint32)
    lens[2222] = 2  # "invalid block data" (crc_util.go:89-91)
    buf, off, lens = oracle.fill_blocks(0x31, len(lens), sizes=lens)
    hc.stamp_blocks(buf, off=off, lens=lens)
    err, bm, fb = hc.multi_verify_blocks(buf, [0, 0], off=off, lens=lens)
    assert fb == 2222 and str(err) == "invalid block data"


def test_multi_stamp_equals_stamp(cuda, hc, oracle):
    n, B = 7_777, 4096
    a = blocks(oracle, n, B, seed=0x12)
    b = a.copy()
    hc.multi_stamp_blocks(a, [0, 0, 0], stride=B, ulen=B)
    hc.stamp_blocks(b, stride=B, ulen=B)
    assert np.array_equal(a, b)
    want = oracle.crc32_blocks(b, stride=B, ulen=B)
    assert np.array_equal(a.reshape(n, B)[:, :4].copy().view(np.uint32).ravel(), want)


def test_dev_multi_shards_equal_one_launch(cuda, hc):
    torch = cuda
    n, B = 100_003, 8192
    buf = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(buf, 0x5EED, stride=B, ulen=B, nblocks=n)
    whole = torch.empty(n, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, whole, stride=B, ulen=B, nblocks=n)
    bounds = hc.shard_plan(n, 3)
    outs, shards = [], []
    for d in range(3):
        lo, hi = int(bounds[d]), int(bounds[d + 1])
        o = torch.empty(hi - lo, dtype=torch.int32, device="cuda")
        outs.append(o)
        shards.append(dict(device=0, buf=buf[lo * B:hi * B], out=o, stride=B, ulen=B, nblocks=hi - lo))
    hc.dev_multi_crc32_blocks(shards)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), whole)


def test_multi_more_devices_than_blocks(cuda, hc, oracle):
    """8 ranges over 5 blocks: the empty ranges do nothing, the others run."""
    n, B = 5, 4096
    buf = blocks(oracle, n, B, seed=0x3)
    want = oracle.crc32_blocks(buf, stride=B, ulen=B)
    assert np.array_equal(hc.multi_crc32_blocks(buf, [0] * 8, stride=B, ulen=B), want)
    err, bm, fb = hc.multi_verify_blocks(buf, [0] * 8, stride=B, ulen=B)
    assert fb == 0 and err is not None  # unstamped blocks fail


def test_multi_pinned_span_dma(cuda, hc, oracle):
    """Pinned records through the span-DMA path of every range's pipeline."""
    torch = cuda
    rng = np.random.default_rng(11)
    lens = rng.integers(64, 65536, 4000).astype(np.uint32)
    host, off, lens = oracle.fill_blocks(0x44, len(lens), sizes=lens)
    pinned = torch.empty(len(host), dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = host
    want = oracle.crc32_blocks(host, off=off, lens=lens)
    got = hc.multi_crc32_blocks(pinned.numpy(), [0, 0, 0], off=off, lens=lens)
    assert np.array_equal(got, want)
