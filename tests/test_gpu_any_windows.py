"""k_crc_any's windows (small batches): 64 messages a window on
large batches, fewer (32 .. 1) when the batch has under 64 per wave, so every
wave gets one.  Batch sizes around every window size, in block mode (off/len
blocks k_crc_grp leaves to the sweep: 1 KiB and misaligned 4 KiB blocks, with
a corrupt block found by verify) and whole-message mode with gaps, out of
order (the stream takes sorted gapped records since round 5; unsorted ones go
to k_crc_any on the device flag, or from 2^14 records to the stream over their
sorted view since round 6), every word against the oracle
(crc_util.go:15-17 / :88-100 per block)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# total waves on MI355X: 256 CUs x 16 = 4096; window 2^w while n < 64 * 4096
NS = [1, 63, 65, 4095, 4097, 8195, 16390, 70001, 140000, 262149]


def u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n", NS)
def test_sweep_blocks_all_window_sizes(cuda, hc, oracle, n):
    torch = cuda
    rng = np.random.default_rng(n)
    # 1 KiB blocks (not a 4 KiB multiple), every 7th a misaligned 4 KiB one
    lens = np.where(np.arange(n) % 7 == 3, 4096, 1024).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 16)
    off += np.uint64(16) + (np.arange(n, dtype=np.uint64) % 7 == 3) * np.uint64(4)
    total = int(off[-1]) + int(lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n)
    torch.cuda.synchronize()
    want = oracle.crc32_blocks(host, off=off, lens=lens, threads=16)
    got = u32(out)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (n, bad[:8])
    # stamp, corrupt one block, verify: the bitmap and first_bad name it
    hc.dev_crc32_blocks(buf, None, off=doff, lens=dlen, nblocks=n, flags=hc.HC_F_STAMP)
    k = int(rng.integers(0, n))
    p = int(off[k]) + 4 + int(rng.integers(0, int(lens[k]) - 4))
    buf[p] ^= 0x20
    bm = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.zeros(1, dtype=torch.int64, device="cuda")
    hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, None, off=doff, lens=dlen, nblocks=n, bad_bitmap=bm, first_bad=fb)
    torch.cuda.synchronize()
    bits = np.unpackbits(u32(bm).view(np.uint8), bitorder="little")[:n]
    assert np.flatnonzero(bits).tolist() == [k] and int(fb.item()) == k


@pytest.mark.parametrize("n", NS)
def test_gapped_messages_all_window_sizes(cuda, hc, oracle, n):
    torch = cuda
    rng = np.random.default_rng(n + 1)
    lens = (64.0 * np.exp(rng.random(n) * np.log(64.0))).astype(np.uint32)  # 64 B - 4 KiB
    lens[::5] = rng.integers(0, 1100, (n + 4) // 5)  # short ones: lane-parallel path
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)  # gaps: not packed
    off += np.uint64(5)
    total = int(off[-1]) + int(lens[-1]) + 64
    p = rng.permutation(n)  # out of order: the stream's fallback
    off, lens = off[p], lens[p]
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    # one record is packed: the stream takes it; from HC_SEG_SORT_MIN records (2^18)
    # the permuted batch is sorted and the stream takes the sorted view (round 6)
    if n >= 1 << 18:
        from test_gpu_seg_sort import sorted_path
        assert hc.seg_path() == sorted_path(buf.data_ptr(), off, lens)
    else:
        assert hc.seg_taken() == (n == 1)
    want = oracle.crc32_messages(host, off, lens, threads=16)
    got = u32(out)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (n, bad[:8])
